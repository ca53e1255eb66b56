# Round 4 A/B: the chain pass's chunk-count scan as one run per thread (build) vs HEAD (build_h).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/ab15
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_synth_parity.py tests/test_cli.py tests/test_dist.py tests/test_records.py tests/test_scale_parity.py tests/test_long_reads.py tests/test_abi.py -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 1
for b in build_h build; do
  SBAM_LIB=$PWD/spark-bam_amd/$b/libsbam.so timeout -k 10 300 python -u tools/bench_kernels.py --size-gb 10 --only check_full --reps 3 > $OUT/kernc_$b.log 2>&1 || exit 2
done
