# Many-contig full check (k_check_bits with the device length table past 4096 contigs): parity, then the 10 GB bench
# at 5000 contigs next to the default line.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/contigs
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_synth_parity.py tests/test_abi.py -x -q -m gpu --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --steps 5 --no-cpu-baseline --e2e-windows 0 --contigs 5000 > $OUT/bench_contigs5000.log 2>&1 || exit 2
timeout -k 10 400 python -u bench.py --steps 5 --no-cpu-baseline --e2e-windows 0 > $OUT/bench_default.log 2>&1 || exit 3
