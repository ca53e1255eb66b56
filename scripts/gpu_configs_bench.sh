# configs[3] / streamed bench lines: loadReads resident at 10 GB, loadReads 100 GB in 10 windows, full-check 30 GB in
# 3 windows (one GPU; window w+1's host staging + H2D overlap window w's kernels)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --workload load-reads --no-cpu-baseline --e2e-windows 0 > gpurun_out/bench_load_reads_10g.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --workload load-reads --size-gb 100 --windows 10 --steps 2 --warmup 1 --no-cpu-baseline --e2e-windows 0 > gpurun_out/bench_load_reads_100g_win10.log 2>&1 || exit 2
timeout -k 10 600 python -u bench.py --size-gb 30 --windows 3 --steps 3 --warmup 1 --no-cpu-baseline --e2e-windows 0 > gpurun_out/bench_fc_30g_win3.log 2>&1 || exit 3
