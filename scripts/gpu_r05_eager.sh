# Eager A/B: parity (eager tests) on the new build, then the check_eager microbench at 10 GB on both builds.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/eager
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_eager_wave.py tests/test_synth_parity.py tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 1
for b in ${LIBS:-build build_e0}; do
  SBAM_LIB=$PWD/spark-bam_amd/$b/libsbam.so timeout -k 10 300 python -u tools/bench_kernels.py --size-gb 10 --only check_eager --reps 5 > $OUT/kern_$b.log 2>&1 || exit 2
done
