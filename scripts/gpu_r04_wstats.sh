# Round 4: decoder + resolver phase attribution (s_memtime per phase, build_stats = -DSBAM_WAVE_STATS), 2 GB.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/wstats
mkdir -p $OUT
timeout -k 10 300 python -u tools/wave_stats.py 2 > $OUT/wave_stats.log 2>&1 || exit 1
