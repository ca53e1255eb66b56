# Round-6 checker changes: GPU parity (long reads, fixtures, synthetic, eager), then k_check_bits A/B on the 10 GB
# short-read workload (build vs build_base) and the long-read bench line.  Output: gpurun_out/r06/chk/${TAG}
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r06/chk/${TAG:-x}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_long_reads.py tests/test_gpu_parity.py tests/test_synth_parity.py tests/test_eager_wave.py} -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 1
for b in ${LIBS:-build build_base build build_base}; do
  SBAM_LIB=$PWD/spark-bam_amd/$b/libsbam.so timeout -k 10 300 python -u tools/bench_kernels.py --size-gb 10 --only ${ONLY:-check_full,check_eager} --reps 5 >> $OUT/kern_$b.log 2>&1 || exit 2
done
if [ -n "$LONG" ]; then
  timeout -k 10 400 python -u bench.py --read-len 0 --e2e-windows 0 --no-cpu-baseline > $OUT/bench_long_full.log 2>&1 || exit 3
  timeout -k 10 400 python -u bench.py --read-len 0 --e2e-windows 0 --workload load-reads --no-cpu-baseline > $OUT/bench_long_load.log 2>&1 || exit 4
fi
