# list-form chain pass: full GPU suite (incl. synthetic + scale verdict diffs), then checker timing at 10 GB
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/ -x -q -m gpu --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_kernels.py --size-gb 10 --only check_full > gpurun_out/kern_chains.log 2>&1 || exit 2
