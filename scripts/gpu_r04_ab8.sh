# Round 4 A/B: full checker tile staging with both 32-B units' loads before the first wait (build) vs the loop
# (build_sh0).  Parity first.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/ab8
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_synth_parity.py tests/test_cli.py -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 1
for b in build_sh0 build; do
  SBAM_LIB=$PWD/spark-bam_amd/$b/libsbam.so timeout -k 10 300 python -u tools/bench_kernels.py --size-gb 10 --only check_full,check_eager --reps 3 > $OUT/kernc_$b.log 2>&1 || exit 2
done
