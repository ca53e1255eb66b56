# lane-per-block resolve (build_old): resolve time vs number of workgroups in flight, 4 GB
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/resgrid
for w in 2048 512 256 128; do
  SBAM_RES_WGS=$w SBAM_LIB=spark-bam_amd/build_old/libsbam.so timeout -k 10 200 python -u tools/bench_kernels.py --size-gb 4 --only inflate --reps 2 > gpurun_out/resgrid/w$w.log 2>&1 || exit 1
done
SBAM_RES_WGS=256 SBAM_LIB=spark-bam_amd/build_old/libsbam.so timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/resgrid/pmc256 -o p -- python3 tools/bench_kernels.py --size-gb 4 --only inflate --reps 1 > gpurun_out/resgrid/pmc256.log 2>&1 || exit 2
