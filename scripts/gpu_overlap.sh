# can scan+inflate (one stream) overlap a full check (another stream)?  build_old = lane-per-block resolve
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
SBAM_LIB=spark-bam_amd/build_old/libsbam.so timeout -k 10 300 python -u tools/overlap_probe.py --size-gb 4 > gpurun_out/overlap4.log 2>&1 || exit 1
SBAM_LIB=spark-bam_amd/build_old/libsbam.so timeout -k 10 400 python -u tools/overlap_probe.py --size-gb 10 > gpurun_out/overlap10.log 2>&1 || exit 2
