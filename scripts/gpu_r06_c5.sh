set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
D=gpurun_out/r06/chk/${TAG:-c5}; mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_long_reads.py -x -q -m gpu --timeout 300 --timeout-method thread > $D/pytest.log 2>&1 || exit 1
for b in ${LIBS:-build build_base build build_base}; do
  SBAM_LIB=$PWD/spark-bam_amd/$b/libsbam.so timeout -k 10 300 python -u tools/bench_kernels.py --size-gb 10 --only check_full --reps 3 >> $D/kern_$b.log 2>&1 || exit 2
done
for b in ${LLIBS:-build}; do
  SBAM_LIB=$PWD/spark-bam_amd/$b/libsbam.so timeout -k 10 300 python -u tools/bench_kernels.py --size-gb 10 --only check_full --reps 3 --read-len 0 >> $D/kern_long_$b.log 2>&1 || exit 3
done
