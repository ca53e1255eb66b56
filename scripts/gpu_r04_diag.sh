# Round 4 A/B: inflate parity on the current build (TokPool arena, resolver distance test, mode-R register
# stores), LDS-staged coalesced token stores (build_cd), next-window register prefetch (build_w1, w3), checker variants (build_c1: record loop unrolled 2,
# build_c2: byte mask without v_mul), and the decoder's phase attribution (build_stats).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/diag2
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_inflate_streams.py tests/test_synth_parity.py -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; echo "pytest exit $rc" >> $OUT/pytest.log; [ $rc -le 1 ] || exit 1
for b in build build_cd build_w1 build_w3; do
  SBAM_LIB=$PWD/spark-bam_amd/$b/libsbam.so timeout -k 10 300 python -u tools/bench_kernels.py --size-gb 10 --only inflate --reps 3 > $OUT/kern_$b.log 2>&1 || exit 2
done
for b in build build_c1 build_c2; do
  SBAM_LIB=$PWD/spark-bam_amd/$b/libsbam.so timeout -k 10 300 python -u tools/bench_kernels.py --size-gb 10 --only check_full,check_eager --reps 3 > $OUT/kernc_$b.log 2>&1 || exit 3
done
timeout -k 10 300 python -u tools/wave_stats.py 2 > $OUT/wave_stats.log 2>&1 || exit 4
