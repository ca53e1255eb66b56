# decode / resolve grid sweep (lanes per block balance), inflate only at 10 GB; plus the synthetic parity test
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_synth_parity.py -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/pytest_synth.log 2>&1 || exit 1
for d in 512 403 448 384 320; do
  echo "dec $d" >> gpurun_out/grid.log
  SBAM_DEC_WGS=$d timeout -k 10 120 python -u tools/bench_kernels.py --size-gb 10 --only inflate --reps 3 >> gpurun_out/grid.log 2>&1 || exit 2
done
for r in 1024 806 768 537; do
  echo "res $r" >> gpurun_out/grid.log
  SBAM_RES_WGS=$r timeout -k 10 120 python -u tools/bench_kernels.py --size-gb 10 --only inflate --reps 3 >> gpurun_out/grid.log 2>&1 || exit 3
done
