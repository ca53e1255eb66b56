# Round 4, second GPU pass: chain-proof skip + WindowPipe fix validated by the split/record/config parity tests;
# resolver A/B (RESOLVE4, far deferral); decoder phase attribution (wave_stats); then the default bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/run2
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_records.py tests/test_configs_scale.py tests/test_long_reads.py tests/test_inflate_streams.py -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 1
for b in build build_r2nd build_r4 build_r4nd; do
  SBAM_LIB=$PWD/spark-bam_amd/$b/libsbam.so timeout -k 10 300 python -u tools/bench_kernels.py --size-gb 10 --only inflate --reps 3 > $OUT/kern_$b.log 2>&1 || exit 2
done
timeout -k 10 300 python -u tools/wave_stats.py 2 > $OUT/wave_stats.log 2>&1 || exit 3
timeout -k 10 500 python -u bench.py > $OUT/bench.log 2>&1 || exit 4
