# A/B of library builds on the inflate microbench at 10 GB: LIBS="build build_x ..." (dirs under spark-bam_amd/)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for b in ${LIBS:-build}; do
  SBAM_LIB=$PWD/spark-bam_amd/$b/libsbam.so timeout -k 10 300 python -u tools/bench_kernels.py --size-gb 10 --only ${ONLY:-inflate} --reps 3 > gpurun_out/ab_$b.log 2>&1 || exit 1
done
