# Round 4 A/B in one call: resolver waits + decoder token pin (build_r0: v2 inflate; build_r1: new resolver, pin 0; build: both) and checker occupancy (build_base: HEAD; build: 26.8 KB LDS, 5 WGs; build_w6: 6 WGs).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/ab45
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests/test_inflate_streams.py tests/test_gpu_parity.py tests/test_synth_parity.py tests/test_cli.py -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 1
for b in build_r0 build_r1 build; do
  SBAM_LIB=$PWD/spark-bam_amd/$b/libsbam.so timeout -k 10 300 python -u tools/bench_kernels.py --size-gb 10 --only inflate --reps 3 > $OUT/kern_$b.log 2>&1 || exit 2
done
for b in build_base build build_w6; do
  SBAM_LIB=$PWD/spark-bam_amd/$b/libsbam.so timeout -k 10 300 python -u tools/bench_kernels.py --size-gb 10 --only check_full --reps 3 > $OUT/kernc_$b.log 2>&1 || exit 3
done
SBAM_LIB=$PWD/spark-bam_amd/build_w6/libsbam.so timeout -k 10 600 python -u -m pytest tests/test_synth_parity.py tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest_w6.log 2>&1 || exit 4
