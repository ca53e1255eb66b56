# Full-step bench over library builds (LIBS: build dirs under spark-bam_amd/), no CPU baseline and no H2D leg.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/lib_bench_ab
mkdir -p $OUT
for b in ${LIBS:-build}; do
  SBAM_LIB=$PWD/spark-bam_amd/$b/libsbam.so timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --e2e-windows 0 > $OUT/bench_$b.log 2>&1 || exit 2
done
