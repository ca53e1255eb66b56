# Round 4 streamed / configs[3] lines: loadReads 10 GB resident, 100 GB through one GPU in 10 windows, and the
# 30 GB full-check in 3 windows (SBAM_PIPE_DEBUG: per-window waits; SBAM_LOG_GROW: any device reallocation).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/stream
mkdir -p $OUT
timeout -k 10 300 python -u bench.py --workload load-reads > $OUT/bench_load_reads.log 2>&1 || exit 1
SBAM_PIPE_DEBUG=1 SBAM_LOG_GROW=1 timeout -k 10 400 python -u bench.py --size-gb 30 --windows 3 --steps 3 --warmup 1 --no-cpu-baseline --e2e-windows 0 > $OUT/bench_fc_30g_win3.log 2>&1 || exit 2
SBAM_LOG_GROW=1 timeout -k 10 500 python -u bench.py --size-gb 100 --windows 10 --workload load-reads --steps 2 --warmup 1 --no-cpu-baseline --e2e-windows 0 > $OUT/bench_load_reads_100g_win10.log 2>&1 || exit 3
