# Round 4 A/B: checker with the name's last-byte-is-0 bit in the first-invalid-op byte (build, SBAM_FBZ=1) vs
# without (build_fbz0): counts parity (fixtures, synthetic) and the kernel microbench at 10 GB.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/ab3
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_synth_parity.py tests/test_cli.py -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 1
for b in build build_fbz0; do
  SBAM_LIB=$PWD/spark-bam_amd/$b/libsbam.so timeout -k 10 300 python -u tools/bench_kernels.py --size-gb 10 --only check_full,check_eager --reps 3 > $OUT/kernc_$b.log 2>&1 || exit 2
done
