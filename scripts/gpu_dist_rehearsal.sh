# rehearse bench.py N=2 through its own rank launcher (two ranks time-sharing the box's one GPU; gloo for the
# small collectives, since RCCL needs one GPU per rank)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python bench.py --gpus 2 --steps 3 --warmup 1 --size-gb 4 --dist-backend gloo --device 0 \
  --no-cpu-baseline --e2e-windows 0 > gpurun_out/bench_n2_rehearsal.log 2>&1 || exit 1
