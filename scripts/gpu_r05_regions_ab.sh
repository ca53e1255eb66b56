# Inflate microbench at 10 GB over builds (LIBS: build dirs; a name ending in :nr runs with SBAM_NO_REGIONS=1).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/regions_ab
mkdir -p $OUT
for v in ${LIBS:-build build:nr build_nopiece:nr build_head}; do
  b=${v%%:*}
  nr=0; [ "$v" != "$b" ] && nr=1
  SBAM_NO_REGIONS=$nr SBAM_LIB=$PWD/spark-bam_amd/$b/libsbam.so timeout -k 10 300 python -u tools/bench_kernels.py --size-gb 10 --only inflate --reps 5 > $OUT/kern_${b}_nr$nr.log 2>&1 || exit 2
done
