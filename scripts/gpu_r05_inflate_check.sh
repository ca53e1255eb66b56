# Inflate parity (streams, fixtures, synthetic every-offset, a 20K-block fuzz corpus) and the inflate microbench at
# 10 GB for the current build (and build_head when present).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/inflate_check
mkdir -p $OUT
SBAM_FUZZ_BLOCKS=20000 timeout -k 10 500 python -u -m pytest tests/test_inflate_streams.py tests/test_synth_parity.py tests/test_inflate_fuzz.py tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_kernels.py --size-gb 10 --only inflate --reps 5 > $OUT/kern.log 2>&1 || exit 2
