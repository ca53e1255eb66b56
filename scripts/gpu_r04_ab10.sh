# Round 4 A/B: resolver see-through (a waiting match copies through the ready match whose output holds its source;
# build) vs none (build_ns).  Parity first; wave stats (rounds per step) with build_stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/ab10
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests/test_inflate_streams.py tests/test_gpu_parity.py tests/test_synth_parity.py -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 1
for b in build_ns build; do
  SBAM_LIB=$PWD/spark-bam_amd/$b/libsbam.so timeout -k 10 300 python -u tools/bench_kernels.py --size-gb 10 --only inflate --reps 3 > $OUT/kern_$b.log 2>&1 || exit 2
done
timeout -k 10 300 python -u tools/wave_stats.py 2 > $OUT/wave_stats.log 2>&1 || exit 3
