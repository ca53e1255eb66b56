# decode symbol slots per step x input prefetch depth: inflate parity + 10 GB inflate timing per variant
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for k in k2p1 k2p2 k2p3 k3p3; do
  export SBAM_LIB=$PWD/spark-bam_amd/build_$k/libsbam.so
  timeout -k 10 300 python -u -m pytest tests/test_inflate_streams.py tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_$k.log 2>&1 || exit 1
  timeout -k 10 300 python -u tools/bench_kernels.py --size-gb 10 --only inflate --reps 3 > gpurun_out/kern_$k.log 2>&1 || exit 2
done
