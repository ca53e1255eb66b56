# Round 4: split_starts' block lookups galloping from the previous split's answer (host; ~1 ms of host time per
# 10 GB step before): split/record parity and the default bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/ab19
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_cli.py tests/test_records.py tests/test_dist.py tests/test_long_reads.py tests/test_cli_blocks.py -x -q -m gpu --timeout 400 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $OUT/bench_default.log 2>&1 || exit 2
