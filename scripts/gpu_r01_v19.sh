# checkpoint v19 (resolve literals after copies): GPU tests, PMC traffic passes, default bench line (+cpu_baseline), kernel-trace stats, load-reads bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit 1
OUT=gpurun_out/pmc_traffic
rm -rf $OUT; mkdir -p $OUT
run() { timeout -s KILL 300 rocprofv3 --pmc $2 --output-format csv -d $OUT/$1 -o p -- python3 tools/bench_kernels.py --size-gb 10 --only inflate,check_full --reps 1 > $OUT/$1.log 2>&1; }
run f "FETCH_SIZE" || exit 2
run w "WRITE_SIZE" || exit 3
python3 tools/traffic_pmc.py $OUT/traffic.json $OUT/f $OUT/w > $OUT/summary.log 2>&1 || exit 4
cp $OUT/traffic.json profiles/r01/traffic.json
timeout -k 10 600 python -u bench.py > gpurun_out/bench_default.log 2>&1 || exit 5
rm -rf gpurun_out/prof_bench
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o p -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_prof.log 2>&1 || exit 6
timeout -k 10 600 python -u bench.py --steps 3 --workload load-reads > gpurun_out/bench_lr.log 2>&1 || exit 7
