# Round 4 A/B: decoder register budget (build_t64 / build_t72: register tokens; build_cp8: 8 checkpoints of 12
# symbols) against the default build, inflate parity on each, kernel microbench at 10 GB.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/ab2
mkdir -p $OUT
for b in build build_t64 build_t72 build_cp8; do
  SBAM_LIB=$PWD/spark-bam_amd/$b/libsbam.so timeout -k 10 300 python -u -m pytest tests/test_inflate_streams.py -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest_$b.log 2>&1 || exit 1
  SBAM_LIB=$PWD/spark-bam_amd/$b/libsbam.so timeout -k 10 300 python -u tools/bench_kernels.py --size-gb 10 --only inflate --reps 3 > $OUT/kern_$b.log 2>&1 || exit 2
done
