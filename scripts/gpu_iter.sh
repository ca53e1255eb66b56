# GPU iteration: parity tests, kernel microbench, 10 GB bench, PMC passes on the checker
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/bench_kernels.py --size-gb 2 > gpurun_out/kern.log 2>&1 || exit 2
timeout -k 10 300 python -u bench.py --size-gb 10 --steps 3 --warmup 1 > gpurun_out/bench_10g.log 2>&1 || exit 3
bash scripts/gpu_pmc.sh build || exit 4
