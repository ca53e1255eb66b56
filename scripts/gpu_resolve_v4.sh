# lane-per-block resolve with 64-B token reads, 64-B output groups, unaligned far loads: parity, timing, traffic
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 240 python -u -m pytest tests/test_inflate_streams.py -x -q -m gpu --timeout 60 --timeout-method thread > gpurun_out/pytest_inflate.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit 2
timeout -k 10 300 python -u tools/bench_kernels.py --size-gb 10 --only inflate --reps 2 > gpurun_out/kern10.log 2>&1 || exit 3
OUT=gpurun_out/pmc_res4
mkdir -p $OUT
run() { timeout -s KILL 150 rocprofv3 --pmc $2 --output-format csv -d $OUT/$1 -o p -- python3 tools/bench_kernels.py --size-gb 4 --only inflate --reps 1 > $OUT/$1.log 2>&1; }
run c "FETCH_SIZE" || exit 4
run d "WRITE_SIZE GRBM_GUI_ACTIVE" || exit 5
