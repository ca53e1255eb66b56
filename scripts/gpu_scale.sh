# verdict diff / CRC / eager-vs-full at scale (4 GB synthetic)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_scale_parity.py -x -v -m gpu --timeout 400 --timeout-method thread > gpurun_out/pytest_scale.log 2>&1 || exit 1
