# streaming windows: sbam_load GPU test, then 30 GB through one GPU in 3 pipelined windows
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_abi.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_load.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --size-gb 30 --windows 3 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_win3.log 2>&1 || exit 2
