# decode / resolve grid re-sweep after v16-v19 (inflate only at 10 GB)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/grid2.log
for r in 1024 896 768 640; do
  echo "res $r" >> gpurun_out/grid2.log
  SBAM_RES_WGS=$r timeout -k 10 120 python -u tools/bench_kernels.py --size-gb 10 --only inflate --reps 3 >> gpurun_out/grid2.log 2>&1 || exit 3
done
for d in 512 448; do
  echo "dec $d" >> gpurun_out/grid2.log
  SBAM_DEC_WGS=$d timeout -k 10 120 python -u tools/bench_kernels.py --size-gb 10 --only inflate --reps 3 >> gpurun_out/grid2.log 2>&1 || exit 2
done
