# Inflate fuzz: the 100K-block test on the product library, then the same corpus tool on the wave-statistics build
# (path counts for the log).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/fuzz
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_inflate_fuzz.py -x -v -s -m gpu --timeout 500 --timeout-method thread > $OUT/pytest_fuzz.log 2>&1 || exit 1
SBAM_LIB=$PWD/spark-bam_amd/build_stats/libsbam.so timeout -k 10 600 python -u tools/inflate_fuzz.py --blocks 100000 > $OUT/fuzz_stats.log 2>&1 || exit 2
