# Round 4: loadReads with the splits' record chains proved from the eager checker's calls (sbam.dist.shard_load
# eager_proof) instead of walked record by record: parity (records tests incl. the eager-bitmap path, the streamed
# configs[3] windows vs the resident walk, dist) and the load-reads bench line (v3 before: 88.1 GB/s, 113.4 ms).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/ab17
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_records.py tests/test_configs_scale.py tests/test_dist.py -x -q -m gpu --timeout 400 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --workload load-reads > $OUT/bench_load_reads.log 2>&1 || exit 2
