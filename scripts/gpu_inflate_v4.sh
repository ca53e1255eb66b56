# Inflate without flat accesses: parity, per-kernel timing, PMC on the inflate kernels
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_inflate_streams.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_inflate.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit 2
timeout -k 10 200 python -u tools/bench_kernels.py --size-gb 2 > gpurun_out/kern.log 2>&1 || exit 3
bash scripts/gpu_pmc_inflate.sh gpurun_out/pmc_inf || exit 4
