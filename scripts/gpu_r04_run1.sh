# Round 4, first GPU pass: the straddle test on the round-3 gate (expected to fail) and the fixed gate, inflate
# parity on both resolver builds with the kernel microbench, the lazy checker timing, then the default bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/run1
mkdir -p $OUT
SBAM_LIB=$PWD/spark-bam_amd/build_old/libsbam.so timeout -k 10 200 python -u -m pytest tests/test_inflate_streams.py -k round_boundary -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest_old_gate.log 2>&1
echo "old gate pytest exit $?" >> $OUT/pytest_old_gate.log
for b in build_res2 build; do
  SBAM_LIB=$PWD/spark-bam_amd/$b/libsbam.so timeout -k 10 400 python -u -m pytest tests/test_inflate_streams.py tests/test_synth_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest_$b.log 2>&1 || exit 1
  SBAM_LIB=$PWD/spark-bam_amd/$b/libsbam.so timeout -k 10 300 python -u tools/bench_kernels.py --size-gb 10 --only inflate --reps 3 > $OUT/kern_$b.log 2>&1 || exit 2
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "lazy" -x -v -s -m gpu --timeout 240 --timeout-method thread > $OUT/pytest_lazy.log 2>&1 || exit 3
timeout -k 10 500 python -u bench.py > $OUT/bench.log 2>&1 || exit 4
timeout -k 10 300 python -u tools/wave_stats.py 2 > $OUT/wave_stats.log 2>&1 || exit 5
