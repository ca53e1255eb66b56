# Round-6: the whole GPU suite on the working tree, then the default bench line and the kernel A/B (build vs
# build_base).  Output: gpurun_out/r06/full/${TAG}
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r06/full/${TAG:-x}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > $OUT/bench_default.log 2>&1 || exit 2
for b in ${LIBS:-build build_base build build_base}; do
  SBAM_LIB=$PWD/spark-bam_amd/$b/libsbam.so timeout -k 10 300 python -u tools/bench_kernels.py --size-gb 10 --only ${ONLY:-check_full} --reps 3 >> $OUT/kern_$b.log 2>&1 || exit 3
done
