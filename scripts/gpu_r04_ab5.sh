# Round 4 A/B: resolver waits.  build: far sources waited on their own path (SBAM_RES_FARWAIT), output stores
# issued before the step's loads (SBAM_RES_EARLYFLUSH), next-step tokens split after the rounds (SBAM_RES_TOKWAIT);
# build_r1: the first only; build_r0: none (the v2 resolver).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/ab5
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_inflate_streams.py tests/test_gpu_parity.py tests/test_synth_parity.py -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 1
for b in build_r0 build_r1 build; do
  SBAM_LIB=$PWD/spark-bam_amd/$b/libsbam.so timeout -k 10 300 python -u tools/bench_kernels.py --size-gb 10 --only inflate --reps 3 > $OUT/kern_$b.log 2>&1 || exit 2
done
