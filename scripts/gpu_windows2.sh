# streaming windows, steady state: 30 GB full-check (3 windows) and the 100 GB loadReads config (10 windows)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --size-gb 30 --windows 3 --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/bench_win3.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --size-gb 100 --windows 10 --workload load-reads --steps 2 --warmup 2 > gpurun_out/bench_100g_lr.log 2>&1 || exit 2
