# SQ instruction/latency counters of the decode + resolve kernels for each library build in LIBS (dirs under
# spark-bam_amd/), one rocprofv3 --pmc pass per build on the 10 GB inflate microbench.  Output: gpurun_out/pmcab/.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/pmcab
mkdir -p $OUT
CTR=${CTR:-"SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS"}
for b in ${LIBS:-build}; do
  SBAM_LIB=$PWD/spark-bam_amd/$b/libsbam.so timeout -s KILL ${PMC_TIMEOUT:-240} rocprofv3 --pmc $CTR --output-format csv -d $OUT/$b -o p -- python3 tools/bench_kernels.py --size-gb 10 --only inflate --reps 1 > $OUT/$b.log 2>&1 || exit 2
done
python3 tools/pmc_ab_summary.py $OUT ${LIBS:-build} > $OUT/summary.log 2>&1 || exit 3
