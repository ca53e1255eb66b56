# long-op pass grouping A/B: parity on the long-op tests, then the full check at 10 GB, short and long reads
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
D=gpurun_out/r06/chk/${TAG:-c9}; mkdir -p $D
for b in build_g4 build_g2; do
  SBAM_LIB=$PWD/spark-bam_amd/$b/libsbam.so timeout -k 10 400 python -u -m pytest tests/test_long_ops.py tests/test_long_reads.py -x -q -m gpu --timeout 300 --timeout-method thread > $D/pytest_$b.log 2>&1 || exit 1
done
for b in build_head build_g4 build_g2 build_head build_g4 build_g2; do
  SBAM_LIB=$PWD/spark-bam_amd/$b/libsbam.so timeout -k 10 300 python -u tools/bench_kernels.py --size-gb 10 --only check_full --reps 3 --read-len 0 >> $D/kern_long_$b.log 2>&1 || exit 2
done
for b in build_head build_g4 build_g2 build_head build_g4 build_g2; do
  SBAM_LIB=$PWD/spark-bam_amd/$b/libsbam.so timeout -k 10 300 python -u tools/bench_kernels.py --size-gb 10 --only check_full --reps 3 >> $D/kern_$b.log 2>&1 || exit 3
done
