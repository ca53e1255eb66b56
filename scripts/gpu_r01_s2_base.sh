# Session-2 baseline: GPU parity tests, smoke, 10 GB bench, rocprofv3 kernel-trace stats of the same bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 2
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 > gpurun_out/bench_10g.log 2>&1 || exit 3
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o bench -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_prof.log 2>&1 || exit 4
