# interior-only k_check instantiation: GPU suite, then checker timing for launch-bound variants
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/ -x -q -m gpu --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit 1
for v in build build_i5 build_i6; do
  echo "$v" >> gpurun_out/check_split.log
  SBAM_LIB=spark-bam_amd/$v/libsbam.so timeout -k 10 200 python -u tools/bench_kernels.py --size-gb 10 --only check_full,check_eager >> gpurun_out/check_split.log 2>&1 || exit 2
done
