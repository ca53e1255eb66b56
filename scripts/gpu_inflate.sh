# inflate-focused check: inflate parity tests, the kernel microbench at 10 GB (decode / resolve ms), and the
# instrumented wave-decoder phase attribution at 2 GB (tools-only build)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_inflate_streams.py tests/test_gpu_parity.py tests/test_synth_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_inflate.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_kernels.py --size-gb 10 --only inflate --reps 3 > gpurun_out/kern_inflate.log 2>&1 || exit 2
if [ -n "$WAVE_STATS" ]; then
  timeout -k 10 300 python -u tools/wave_stats.py 2 > gpurun_out/wave_stats.log 2>&1 || exit 3
fi
