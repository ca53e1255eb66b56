# Round 4 A/B: the BGZF candidate scan with P positions per thread and iteration and one barrier per iteration
# without candidates (k_scan_slots_wide<P>: build = P 64, build_s32, build_s16) vs round 4's k_scan_slots (build_s0:
# 16 positions, three barriers per iteration).  Scan / block-table parity of each form first.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/ab23
mkdir -p $OUT
for b in build build_s32 build_s16; do
  SBAM_LIB=$PWD/spark-bam_amd/$b/libsbam.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_inflate_streams.py tests/test_cli_blocks.py tests/test_synth_parity.py -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest_$b.log 2>&1 || exit 1
done
for b in build_s0 build build_s32 build_s16 build_s0; do
  SBAM_LIB=$PWD/spark-bam_amd/$b/libsbam.so timeout -k 10 300 python -u tools/bench_kernels.py --size-gb 10 --only scan --reps 5 > $OUT/kern_$b.log 2>&1 || exit 2
done
