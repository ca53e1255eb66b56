# Round 4 A/B: compute-splits' per-split popcounts with 8 bitmap words in flight per thread (build) vs HEAD
# (build_h): the bench step's `records` time.  Parity first.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/ab16
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_records.py tests/test_gpu_parity.py tests/test_cli.py tests/test_synth_parity.py tests/test_dist.py -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 1
for b in build_h build; do
  SBAM_LIB=$PWD/spark-bam_amd/$b/libsbam.so timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --e2e-windows 0 > $OUT/bench_$b.log 2>&1 || exit 2
done
