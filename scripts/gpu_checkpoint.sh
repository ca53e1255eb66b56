# checkpoint: GPU tests, smoke, default bench line (cpu_baseline, e2e_h2d, copy peak), kernel-trace stats, then the
# PMC passes (traffic + SQ counters) of the same sources
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || exit 2
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o p -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --e2e-windows 0 > gpurun_out/bench_prof.log 2>&1 || exit 4
ONLY=inflate,check_full bash scripts/gpu_pmc.sh || exit 5
timeout -k 10 600 python -u bench.py > gpurun_out/bench_default.log 2>&1 || exit 3
