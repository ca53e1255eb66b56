# k_check launch-bounds sweep (workgroups per CU the VGPR budget is sized for): checker timing at 10 GB
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in build build_w3 build_w5 build_w6; do
  echo "$v" >> gpurun_out/check_wgs.log
  SBAM_LIB=spark-bam_amd/$v/libsbam.so timeout -k 10 200 python -u tools/bench_kernels.py --size-gb 10 --only check_full,check_eager >> gpurun_out/check_wgs.log 2>&1 || exit 1
done
