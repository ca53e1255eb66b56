# Round-6 final sources: the other bench lines (loadReads, zlib levels 0/1, real data) re-measured after the host-path pass.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/lines
mkdir -p $OUT
timeout -k 10 400 python -u bench.py --workload load-reads --e2e-windows 0 --no-cpu-baseline > $OUT/bench_load_reads.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --level 1 --e2e-windows 0 --no-cpu-baseline > $OUT/bench_level1.log 2>&1 || exit 2
timeout -k 10 400 python -u bench.py --level 0 --e2e-windows 0 --no-cpu-baseline > $OUT/bench_level0.log 2>&1 || exit 3
timeout -k 10 400 python -u bench.py --real --e2e-windows 0 --no-cpu-baseline > $OUT/bench_real.log 2>&1 || exit 4
