# GPU round: parity tests then checker/inflate timing at 2 GB for several inflate lane counts
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit 1
for L in 16384 32768 65536 131072; do
  SBAM_INFLATE_LANES=$L timeout -k 10 200 python -u bench.py --size-gb 2 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_lanes_$L.log 2>&1 || exit 2
done
