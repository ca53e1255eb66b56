# Resolver A/B: inflate parity subset on the variant build, then the inflate microbench at 10 GB over LIBS.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/res_ab
mkdir -p $OUT
V=${VARIANT:-build_ringw}
SBAM_LIB=$PWD/spark-bam_amd/$V/libsbam.so SBAM_FUZZ_BLOCKS=5000 timeout -k 10 500 python -u -m pytest tests/test_inflate_streams.py tests/test_synth_parity.py tests/test_inflate_fuzz.py -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest_$V.log 2>&1 || exit 1
for b in ${LIBS:-build_ringw build build_ringw build}; do
  SBAM_LIB=$PWD/spark-bam_amd/$b/libsbam.so timeout -k 10 300 python -u tools/bench_kernels.py --size-gb 10 --only inflate --reps 5 > $OUT/kern_$b.log 2>&1 || exit 2
done
