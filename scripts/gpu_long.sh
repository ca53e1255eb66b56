# long-read config parity on the GPU
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_long_reads.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_long.log 2>&1 || exit 1
