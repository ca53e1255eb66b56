# Round 4 A/B: k_eager with per-wave survivor queues (no workgroup barrier between the prefilter and the bitmap
# write-out; build) vs one workgroup queue (build_wq0).  Eager parity first.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/ab20
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_synth_parity.py tests/test_cli.py tests/test_records.py -x -q -m gpu --timeout 400 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 1
for b in build_wq0 build; do
  SBAM_LIB=$PWD/spark-bam_amd/$b/libsbam.so timeout -k 10 300 python -u tools/bench_kernels.py --size-gb 10 --only check_eager --reps 5 > $OUT/kerne_$b.log 2>&1 || exit 2
done
SBAM_LIB=$PWD/spark-bam_amd/build/libsbam.so timeout -k 10 400 python -u bench.py --no-cpu-baseline --e2e-windows 0 > $OUT/bench_default.log 2>&1 || exit 3
