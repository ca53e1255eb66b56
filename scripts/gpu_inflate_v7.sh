# decode v3 (2 waves/SIMD, interleaved 320-B slices, register input window): parity + timing
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_inflate_streams.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_inflate.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit 2
timeout -k 10 200 python -u tools/bench_kernels.py --size-gb 2 --only inflate > gpurun_out/kern2.log 2>&1 || exit 3
timeout -k 10 300 python -u tools/bench_kernels.py --size-gb 10 --only inflate --reps 2 > gpurun_out/kern10.log 2>&1 || exit 4
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_10g.log 2>&1 || exit 5
