# A/B of library builds (LIBS = dirs under spark-bam_amd/): inflate parity tests (unless NOTEST) and the kernel
# microbench at 10 GB (ONLY = stage list) for each; optional PMC pass (PMC=1) on the inflate kernels.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/ab
mkdir -p $OUT
for b in ${LIBS:-build}; do
  export SBAM_LIB=$PWD/spark-bam_amd/$b/libsbam.so
  if [ -z "$NOTEST" ]; then
    timeout -k 10 300 python -u -m pytest ${TESTS:-tests/test_inflate_streams.py tests/test_synth_parity.py} -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest_$b.log 2>&1 || exit 1
  fi
  timeout -k 10 300 python -u tools/bench_kernels.py --size-gb 10 --only ${ONLY:-inflate} --reps 3 > $OUT/kern_$b.log 2>&1 || exit 2
  if [ -n "$PMC" ]; then
    timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS --output-format csv -d $OUT/pmc_$b -o p -- python3 tools/bench_kernels.py --size-gb 10 --only inflate --reps 1 > $OUT/pmc_$b.log 2>&1 || exit 3
  fi
done
