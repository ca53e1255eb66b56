# loadBamIntervals GPU tests, then the whole GPU suite
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_intervals.py tests/test_abi.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_intervals.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit 2
