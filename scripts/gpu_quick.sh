# GPU quick iteration: parity tests + per-kernel microbenchmark at 2 GB
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/bench_kernels.py --size-gb 2 > gpurun_out/kern.log 2>&1 || exit 2
