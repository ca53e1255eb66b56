# Round-6 A/B: parity subset on the candidate build (spark-bam_amd/build), then the inflate microbench at 10 GB
# alternating candidate and baseline (spark-bam_amd/build_base).  Output: gpurun_out/r06/ab/
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r06/ab/${TAG:-x}
mkdir -p $OUT
SBAM_FUZZ_BLOCKS=${FUZZ:-20000} timeout -k 10 500 python -u -m pytest ${TESTS:-tests/test_inflate_streams.py tests/test_synth_parity.py tests/test_inflate_fuzz.py} -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 1
for b in ${LIBS:-build build_base build build_base}; do
  SBAM_LIB=$PWD/spark-bam_amd/$b/libsbam.so timeout -k 10 300 python -u tools/bench_kernels.py --size-gb 10 --only ${ONLY:-inflate} --reps 5 >> $OUT/kern_$b.log 2>&1 || exit 2
done
