# Round-6 long reads (configs[4]): parity, the full-check and loadReads bench lines, a kernel trace of the full-check
# line, and configs[2]'s shape over long reads (4 ranks over gloo on the one GPU: halo retries).  Output:
# gpurun_out/r06/long/${TAG}
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r06/long/${TAG:-x}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_long_reads.py tests/test_gpu_parity.py tests/test_synth_parity.py -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --read-len 0 --e2e-windows 0 > $OUT/bench_long_full.log 2>&1 || exit 2
timeout -k 10 400 python -u bench.py --read-len 0 --e2e-windows 0 --workload load-reads > $OUT/bench_long_load.log 2>&1 || exit 3
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o long -- python3 bench.py --read-len 0 --e2e-windows 0 --no-cpu-baseline --steps 3 > $OUT/prof.log 2>&1 || exit 4
timeout -k 10 500 python -u bench.py --read-len 0 --gpus 4 --size-gb 2 --dist-backend gloo --device 0 --e2e-windows 0 --no-cpu-baseline > $OUT/bench_long_n4_gloo.log 2>&1 || exit 5
