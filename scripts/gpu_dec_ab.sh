# A/B over build directories given as arguments (inflate parity + 10 GB inflate timing each)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in "$@"; do
  export SBAM_LIB=$PWD/spark-bam_amd/$v/libsbam.so
  timeout -k 10 300 python -u -m pytest tests/test_inflate_streams.py tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_$v.log 2>&1 || exit 1
  timeout -k 10 300 python -u tools/bench_kernels.py --size-gb 10 --only inflate --reps 3 > gpurun_out/kern_$v.log 2>&1 || exit 2
done
