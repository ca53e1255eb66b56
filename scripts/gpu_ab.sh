# Kernel A/B: parity subset (TESTS) on the first library build of LIBS, then the kernel microbench (ONLY stages,
# 10 GB) on every build of LIBS (dirs under spark-bam_amd/); WAVE_STATS=1 adds the instrumented decoder's phase
# attribution (build_stats).  Output: gpurun_out/ab/.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/ab
mkdir -p $OUT
LIBS=${LIBS:-build}
first=${LIBS%% *}
if [ -n "$TESTS" ]; then
  SBAM_LIB=$PWD/spark-bam_amd/$first/libsbam.so timeout -k 10 400 python -u -m pytest $TESTS -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest_$first.log 2>&1 || exit 1
fi
for b in $LIBS; do
  SBAM_LIB=$PWD/spark-bam_amd/$b/libsbam.so timeout -k 10 300 python -u tools/bench_kernels.py --size-gb 10 --only ${ONLY:-inflate} --reps 3 > $OUT/kern_$b.log 2>&1 || exit 2
done
if [ -n "$WAVE_STATS" ]; then
  timeout -k 10 300 python -u tools/wave_stats.py 2 > $OUT/wave_stats.log 2>&1 || exit 3
fi
