# record decode parity (bitmap proof + walk), the full GPU suite, then the load-reads and streamed benches
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_records.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_records.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit 2
timeout -k 10 600 python -u bench.py --steps 3 --no-cpu-baseline > gpurun_out/bench_fc.log 2>&1 || exit 3
timeout -k 10 600 python -u bench.py --steps 3 --workload load-reads > gpurun_out/bench_lr.log 2>&1 || exit 4
timeout -k 10 900 python -u bench.py --steps 2 --warmup 1 --size-gb 30 --windows 3 --no-cpu-baseline > gpurun_out/bench_fc_win3.log 2>&1 || exit 5
