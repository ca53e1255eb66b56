# resolve A/B: inflate parity tests, then the inflate microbench at 10 GB for each ring size (SBAM_RES_RB)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_inflate_streams.py tests/test_gpu_parity.py tests/test_synth_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_inflate.log 2>&1 || exit 1
for rb in ${RBS:-13 14}; do
  SBAM_RES_RB=$rb timeout -k 10 300 python -u tools/bench_kernels.py --size-gb 10 --only inflate --reps 3 > gpurun_out/kern_inflate_rb$rb.log 2>&1 || exit 2
done
if [ -n "$WAVE_STATS" ]; then
  timeout -k 10 300 python -u tools/wave_stats.py 2 > gpurun_out/wave_stats.log 2>&1 || exit 3
fi
