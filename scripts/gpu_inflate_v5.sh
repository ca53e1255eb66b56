# Parked header builds: parity, then inflate timing for park thresholds 8/16/32
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_inflate_streams.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_inflate.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit 2
for v in build build_pm8 build_pm32; do
  SBAM_LIB=spark-bam_amd/$v/libsbam.so timeout -k 10 200 python -u tools/bench_kernels.py --size-gb 2 --only inflate > gpurun_out/kern_$v.log 2>&1 || exit 3
done
bash scripts/gpu_pmc_inflate.sh gpurun_out/pmc_inf5 || exit 4
