# Round 4 A/B: k_eager at 8 waves per SIMD (__launch_bounds__(256, 8): 59 VGPRs) and one barrier less per tile
# (build) vs HEAD (build_e0: 71 VGPRs, 7 waves).  Eager parity first.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/ab11
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_synth_parity.py tests/test_cli.py -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 1
for b in build_e0 build; do
  SBAM_LIB=$PWD/spark-bam_amd/$b/libsbam.so timeout -k 10 300 python -u tools/bench_kernels.py --size-gb 10 --only check_eager --reps 3 > $OUT/kerne_$b.log 2>&1 || exit 2
done
