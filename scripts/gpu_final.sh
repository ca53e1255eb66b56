# Round-end evidence in two calls (PART=1: parity + smoke + default bench + kernel trace; PART=2: PMC passes, the
# default bench again with that traffic (bench.py reads profiles/*/traffic.json of the same sources), and the
# load-reads / streamed bench lines).  Output: gpurun_out/final/ (copy what is judged into profiles/<round>/).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/final
mkdir -p $OUT
if [ "${PART:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests/ -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit 1
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 2
  timeout -k 10 400 python -u bench.py > $OUT/bench_default.log 2>&1 || exit 3
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_bench -o p -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --e2e-windows 0 > $OUT/bench_prof.log 2>&1 || exit 4
else
  ONLY=scan,inflate,check_full,check_eager bash scripts/gpu_pmc.sh || exit 5
  mkdir -p profiles/final_tmp && cp gpurun_out/pmc/traffic.json profiles/final_tmp/traffic.json || exit 5
  timeout -k 10 400 python -u bench.py > $OUT/bench_default_traffic.log 2>&1 || exit 9
  timeout -k 10 300 python -u bench.py --workload load-reads > $OUT/bench_load_reads.log 2>&1 || exit 6
  timeout -k 10 400 python -u bench.py --size-gb 100 --windows 10 --workload load-reads --steps 2 --warmup 1 --no-cpu-baseline --e2e-windows 0 > $OUT/bench_load_reads_100g_win10.log 2>&1 || exit 7
  timeout -k 10 300 python -u bench.py --size-gb 30 --windows 3 --steps 2 --warmup 1 --no-cpu-baseline --e2e-windows 0 > $OUT/bench_fc_30g_win3.log 2>&1 || exit 8
fi
