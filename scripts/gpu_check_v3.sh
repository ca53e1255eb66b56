# Checker with class bitmaps: parity, per-kernel timing at 10 GB, bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit 2
timeout -k 10 300 python -u tools/bench_kernels.py --size-gb 10 --only check_full,check_eager --reps 2 > gpurun_out/kern10_check.log 2>&1 || exit 4
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_10g.log 2>&1 || exit 5
