# decoder phase attribution (instrumented tools-only builds): HEAD's build_stats_head vs the working tree's build_stats
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
SBAM_LIB=$PWD/spark-bam_amd/build_stats_head/libsbam.so timeout -k 10 300 python -u tools/wave_stats.py 2 > gpurun_out/wave_stats_head.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/wave_stats.py 2 > gpurun_out/wave_stats.log 2>&1 || exit 2
