# HBM traffic of the lane-per-block resolve kernel (committed version, build_old) at 4 GB
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/pmc_res_old
mkdir -p $OUT
run() { SBAM_LIB=spark-bam_amd/build_old/libsbam.so timeout -s KILL 150 rocprofv3 --pmc $2 --output-format csv -d $OUT/$1 -o p -- python3 tools/bench_kernels.py --size-gb 4 --only inflate --reps 1 > $OUT/$1.log 2>&1; }
run c "FETCH_SIZE" || exit 3
run d "WRITE_SIZE GRBM_GUI_ACTIVE" || exit 4
run e "TCC_HIT_sum TCC_MISS_sum SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" || exit 5
