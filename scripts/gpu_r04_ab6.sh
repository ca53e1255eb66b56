# Round 4 diagnostic: the decoder's register-token stores done twice (build_dd, SBAM_DUMP_REPS=2) vs once, and
# the phase attribution of the current decoder / resolver (build_stats).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/ab6
mkdir -p $OUT
for b in build build_dd; do
  SBAM_LIB=$PWD/spark-bam_amd/$b/libsbam.so timeout -k 10 300 python -u tools/bench_kernels.py --size-gb 10 --only inflate --reps 3 > $OUT/kern_$b.log 2>&1 || exit 2
done
timeout -k 10 300 python -u tools/wave_stats.py 2 > $OUT/wave_stats.log 2>&1 || exit 3
