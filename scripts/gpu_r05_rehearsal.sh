# configs[2]'s 8-process shape rehearsed on one GPU: 8 ranks through torch.distributed.run
# (gloo collectives, every rank on GPU 0, 3.75 GB each = a 30 GB file), then one process over the same 30 GB file in
# 3 windows; their Counts / split digests must agree.  A rehearsal of the launcher and the gather, not scaling.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/rehearsal
mkdir -p $OUT
timeout -k 10 700 python -u bench.py --gpus 8 --size-gb 3.75 --dist-backend gloo --device 0 --steps 2 --warmup 1 --no-cpu-baseline --e2e-windows 0 > $OUT/bench_n8_gloo_1gpu.log 2>&1 || exit 1
timeout -k 10 500 python -u bench.py --size-gb 30 --windows 3 --steps 1 --warmup 1 --no-cpu-baseline --e2e-windows 0 > $OUT/bench_30g_win3.log 2>&1 || exit 2
