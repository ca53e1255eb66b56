# session-4 re-entry check: GPU parity tests + default bench line on the rebuilt tree
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/bench_default.log 2>&1 || exit 5
