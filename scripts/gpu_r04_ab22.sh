# Round 4 A/B: k_eager staging 64 B past the tile instead of 768 (build_h64: 8.5 % fewer bytes read), the same with
# the next tile by LDS DMA into a second window (build_dma: no prefetch VGPRs, one barrier less; LDS lens 512,
# queue 1024; build_dma8: lens 256, queue 512) vs HEAD (build).  Eager parity of each form first.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/ab22
mkdir -p $OUT
for b in build_h64 build_dma build_dma8; do
  SBAM_LIB=$PWD/spark-bam_amd/$b/libsbam.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_records.py tests/test_long_reads.py -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest_$b.log 2>&1 || exit 1
done
for b in build build_h64 build_dma build_dma8; do
  SBAM_LIB=$PWD/spark-bam_amd/$b/libsbam.so timeout -k 10 300 python -u tools/bench_kernels.py --size-gb 10 --only check_eager --reps 3 > $OUT/kerne_$b.log 2>&1 || exit 2
done
