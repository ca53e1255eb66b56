# GPU test subset (TESTS = pytest paths, default the whole -m gpu suite), then optional extras:
# WAVE_STATS=1 → the instrumented decoder's phase attribution (build_stats); KERN=stage list → kernel microbench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest ${TESTS:-tests} -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/pytest.log 2>&1 || exit 1
if [ -n "$WAVE_STATS" ]; then
  timeout -k 10 300 python -u tools/wave_stats.py 2 > gpurun_out/wave_stats.log 2>&1 || exit 2
fi
if [ -n "$KERN" ]; then
  timeout -k 10 300 python -u tools/bench_kernels.py --size-gb 10 --only $KERN --reps 3 > gpurun_out/kern.log 2>&1 || exit 3
fi
