# wave decoder phase attribution (tools-only instrumented build) + the product build's inflate microbench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/wave_stats.py 2 > gpurun_out/wave_stats.log 2>&1 || exit 1
