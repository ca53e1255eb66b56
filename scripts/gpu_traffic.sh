# tests, PMC traffic passes on the bench workload (10 GB), then the bench line that reads them
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out profiles/r01
timeout -k 10 400 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit 1
OUT=gpurun_out/pmc_traffic
mkdir -p $OUT
run() { timeout -s KILL 300 rocprofv3 --pmc $2 --output-format csv -d $OUT/$1 -o p -- python3 tools/bench_kernels.py --size-gb 10 --only inflate,check_full --reps 1 > $OUT/$1.log 2>&1; }
run f "FETCH_SIZE" || exit 2
run w "WRITE_SIZE" || exit 3
python3 tools/traffic_pmc.py $OUT/traffic.json $OUT/f $OUT/w > $OUT/summary.log 2>&1 || exit 4  # copy into profiles/<round>/ to use it
timeout -k 10 600 python -u bench.py --no-cpu-baseline > gpurun_out/bench_traffic.log 2>&1 || exit 5
