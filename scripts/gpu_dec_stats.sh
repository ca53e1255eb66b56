set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
SBAM_LIB=spark-bam_amd/build_stats/libsbam.so timeout -k 10 300 python -u tools/decode_stats.py --size-gb 10 > gpurun_out/dec_stats10.log 2>&1 || exit 1
SBAM_LIB=spark-bam_amd/build_stats/libsbam.so timeout -k 10 300 python -u tools/decode_stats.py --size-gb 1 > gpurun_out/dec_stats1.log 2>&1 || exit 2
