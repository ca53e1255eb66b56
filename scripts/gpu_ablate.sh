# checker ablation timings (A/B on one box) + counter list
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > gpurun_out/counters.txt 2>&1
for v in build build_a1 build_a2 build_a3 build_a4 build; do
  SBAM_LIB=spark-bam_amd/$v/libsbam.so timeout -k 10 120 python -u tools/bench_kernels.py --size-gb 1 --only check_full,check_eager >> gpurun_out/ablate.log 2>&1 || exit 1
  echo "^ $v" >> gpurun_out/ablate.log
done
