# checker: interior classify (one-hot key planes, no range checks): parity + 10 GB kernel timing
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_kernels.py --size-gb 10 --only check_full,check_eager --reps 3 > gpurun_out/kern10_check.log 2>&1 || exit 2
