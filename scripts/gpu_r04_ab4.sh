# Round 4 A/B: full checker at 6 workgroups per CU.  build: the byte==1 plane dropped (l_read_name == 1 tested per
# position) and the workgroup totals over the planes after the last tile (LDS 28.2 -> 26.8 KB), 5 workgroups;
# build_w6: the same at __launch_bounds__(256, 6) (80 VGPRs, 6 spilled); build_base: HEAD.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/ab4
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_synth_parity.py tests/test_cli.py -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 1
SBAM_LIB=$PWD/spark-bam_amd/build_w6/libsbam.so timeout -k 10 600 python -u -m pytest tests/test_synth_parity.py tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest_w6.log 2>&1 || exit 2
for b in build_base build build_w6; do
  SBAM_LIB=$PWD/spark-bam_amd/$b/libsbam.so timeout -k 10 300 python -u tools/bench_kernels.py --size-gb 10 --only check_full --reps 3 > $OUT/kernc_$b.log 2>&1 || exit 3
done
