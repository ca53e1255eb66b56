# Round-4 first call: the ADVICE straddle test against the round-3 gate (expected to fail) and the fixed gate,
# the inflate parity tests, then the kernel microbench baseline at 10 GB.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r04base
mkdir -p $OUT
SBAM_LIB=$PWD/spark-bam_amd/build_old/libsbam.so timeout -k 10 200 python -u -m pytest tests/test_inflate_streams.py -k round_boundary -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest_old_gate.log 2>&1
echo "old gate pytest exit $?" >> $OUT/pytest_old_gate.log
timeout -k 10 300 python -u -m pytest tests/test_inflate_streams.py -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest_inflate.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_kernels.py --size-gb 10 --only inflate,check_full,check_eager --reps 3 > $OUT/kern.log 2>&1 || exit 2
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "lazy" -x -v -s -m gpu --timeout 240 --timeout-method thread > $OUT/pytest_lazy.log 2>&1 || exit 3
