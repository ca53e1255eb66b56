# Round 5, first GPU call: the whole -m gpu suite, then the loadReads line with the forced chain proof.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r05a
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --workload load-reads --steps 3 --no-cpu-baseline > $OUT/bench_load_reads.log 2>&1 || exit 2
