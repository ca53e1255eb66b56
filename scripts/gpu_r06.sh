# Round-6 GPU steps (STAGE=a: the changed paths' tests + the pinned headline + the --level / --real lines).
# Output: gpurun_out/r06/ (copy what is judged into profiles/r06/).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r06/${STAGE:-a}
mkdir -p $OUT
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu"
case "${STAGE:-a}" in
a)
  timeout -k 10 600 $T tests/test_inflate_streams.py tests/test_records.py tests/test_eager_wave.py tests/test_abi.py > $OUT/pytest.log 2>&1 || exit 1
  timeout -k 10 400 python -u bench.py > $OUT/bench_default.log 2>&1 || exit 2
  timeout -k 10 300 python -u bench.py --level 0 --e2e-windows 0 > $OUT/bench_level0.log 2>&1 || exit 3
  timeout -k 10 300 python -u bench.py --level 1 --e2e-windows 0 > $OUT/bench_level1.log 2>&1 || exit 4
  timeout -k 10 300 python -u bench.py --real --e2e-windows 0 > $OUT/bench_real.log 2>&1 || exit 5
  ;;
b)  # configs[4] long reads: full-check and loadReads lines at 10 GB, then 4 ranks over gloo on the one GPU (halo retries)
  timeout -k 10 400 python -u bench.py --read-len 0 --e2e-windows 0 > $OUT/bench_long_full.log 2>&1 || exit 1
  timeout -k 10 400 python -u bench.py --read-len 0 --e2e-windows 0 --workload load-reads > $OUT/bench_long_load.log 2>&1 || exit 2
  timeout -k 10 500 python -u bench.py --read-len 0 --gpus 4 --size-gb 2 --dist-backend gloo --device 0 --e2e-windows 0 --no-cpu-baseline > $OUT/bench_long_n4_gloo.log 2>&1 || exit 3
  ;;
esac
