# Round 4 A/B: the decoder at 3 waves per SIMD (163 VGPRs, no spills; build_w3), the same with 96 register tokens
# (build_w3t96), vs 4 waves with 20 spilled VGPRs (build).  Inflate parity of the new forms first.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/ab21
mkdir -p $OUT
for b in build_w3 build_w3t96; do
  SBAM_LIB=$PWD/spark-bam_amd/$b/libsbam.so timeout -k 10 600 python -u -m pytest tests/test_inflate_streams.py tests/test_synth_parity.py -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest_$b.log 2>&1 || exit 1
done
for b in build build_w3 build_w3t96; do
  SBAM_LIB=$PWD/spark-bam_amd/$b/libsbam.so timeout -k 10 300 python -u tools/bench_kernels.py --size-gb 10 --only inflate --reps 3 > $OUT/kern_$b.log 2>&1 || exit 2
done
