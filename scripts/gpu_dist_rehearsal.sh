# rehearse bench.py N=2 (two ranks time-sharing the box's one GPU; gloo for the small collectives)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --size-gb 4 --dist-backend gloo --device 0 \
  > gpurun_out/bench_n2_rehearsal.log 2>&1 || exit 1
