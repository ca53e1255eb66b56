# configs[2]/[3] tests on one GPU (8-shard full-check at 4 GB, streamed windows, world-2 GpuShard over gloo)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_configs_scale.py tests/test_dist.py -x -v -m gpu --timeout 400 --timeout-method thread > gpurun_out/pytest_configs.log 2>&1
