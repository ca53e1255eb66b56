# Round 4 A/B: BGZF scan with the next iteration's 32 B loaded before the current candidates are ranked (build)
# vs not (build_sp0).  Parity first.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/ab12
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_inflate_streams.py tests/test_gpu_parity.py tests/test_synth_parity.py tests/test_cli_blocks.py -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 1
for b in build_sp0 build; do
  SBAM_LIB=$PWD/spark-bam_amd/$b/libsbam.so timeout -k 10 300 python -u tools/bench_kernels.py --size-gb 10 --only scan --reps 5 > $OUT/kerns_$b.log 2>&1 || exit 2
done
