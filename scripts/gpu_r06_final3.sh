# Round-6 final sources (block table offsets on the device, its host copy on a side stream; split counts from the PASS0 list, host copy before the result reads, galloped split positions): GPU suite, smoke, PMC traffic of these sources, the default bench
# with that traffic, a kernel trace, and the long-read line.  Output: gpurun_out/final3/
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/final3
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/ -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 2
ONLY=scan,inflate,check_full,check_eager bash scripts/gpu_pmc.sh || exit 3
mkdir -p profiles/final_tmp && cp gpurun_out/pmc/traffic.json profiles/final_tmp/traffic.json || exit 4
timeout -k 10 400 python -u bench.py > $OUT/bench_default_traffic.log 2>&1 || exit 5
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_bench -o p -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --e2e-windows 0 > $OUT/bench_prof.log 2>&1 || exit 6
timeout -k 10 400 python -u bench.py --read-len 0 --e2e-windows 0 > $OUT/bench_long_full.log 2>&1 || exit 7
