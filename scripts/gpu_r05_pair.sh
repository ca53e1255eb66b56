# Decoder A/B: two symbols per phase-A step (build) vs one (build_p0): inflate parity on the new build (streams,
# fixtures, synthetic every-offset, a 20K-block fuzz corpus), then the inflate microbench at 10 GB on both.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/pair
mkdir -p $OUT
SBAM_FUZZ_BLOCKS=20000 timeout -k 10 500 python -u -m pytest tests/test_inflate_streams.py tests/test_synth_parity.py tests/test_inflate_fuzz.py tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 1
for b in ${LIBS:-build build_p0}; do
  SBAM_LIB=$PWD/spark-bam_amd/$b/libsbam.so timeout -k 10 300 python -u tools/bench_kernels.py --size-gb 10 --only inflate --reps 3 > $OUT/kern_$b.log 2>&1 || exit 2
done
