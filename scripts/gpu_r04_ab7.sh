# Round 4 A/B: decoder window staging — all five loads before one wait (build, registers), LDS DMA
# (build_su2, global_load_lds_dwordx4), the load-wait-store loop (build_su0).  Parity of both new forms first.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/ab7
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_inflate_streams.py tests/test_synth_parity.py -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 1
SBAM_LIB=$PWD/spark-bam_amd/build_su2/libsbam.so timeout -k 10 600 python -u -m pytest tests/test_inflate_streams.py tests/test_synth_parity.py -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest_su2.log 2>&1 || exit 2
for b in build_su0 build build_su2; do
  SBAM_LIB=$PWD/spark-bam_amd/$b/libsbam.so timeout -k 10 300 python -u tools/bench_kernels.py --size-gb 10 --only inflate --reps 3 > $OUT/kern_$b.log 2>&1 || exit 3
done
