# Round 4 diagnostic: the resolver with every far-copy load redirected to a cache-resident 4 KiB (build_fh,
# SBAM_DIAG_FARHOT=1, wrong output — timing only) vs build: what the far sources' memory traffic costs.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/ab9
mkdir -p $OUT
for b in build build_fh; do
  SBAM_LIB=$PWD/spark-bam_amd/$b/libsbam.so timeout -k 10 300 python -u tools/bench_kernels.py --size-gb 10 --only inflate --reps 3 > $OUT/kern_$b.log 2>&1 || exit 2
done
