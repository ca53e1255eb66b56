# GPU round: parity tests, smoke, a small and a 10 GB bench (each step time-limited; stop at first failure)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py --size-gb 0.5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_small.log 2>&1 && \
timeout -k 10 400 python -u bench.py --size-gb 10 --steps 3 --warmup 1 > gpurun_out/bench_10g.log 2>&1
echo EXIT $? >> gpurun_out/bench_10g.log
