# kernel microbench at 10 GB (ONLY=stage list) after the checker parity tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_synth_parity.py tests/test_configs_scale.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/pytest_kern.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_kernels.py --size-gb 10 --only ${ONLY:-check_full,check_eager} --reps 3 > gpurun_out/kern.log 2>&1 || exit 2
