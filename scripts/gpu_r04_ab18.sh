# Round 4: loadReads' record columns with one block search per wave (each lane steps forward from it) and the split
# offsets 4 bitmap words per thread and round: parity (records incl. long reads, streamed configs[3]) and the
# load-reads bench line (before: 96.7 GB/s, load_records 4.66 ms).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/ab18
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_records.py tests/test_long_reads.py tests/test_configs_scale.py tests/test_intervals.py -x -q -m gpu --timeout 400 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --workload load-reads > $OUT/bench_load_reads.log 2>&1 || exit 2
