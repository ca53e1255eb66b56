# PMC passes on the two inflate kernels (scan + inflate microbenchmark, 1 GB); one counter group per run
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=${1:-gpurun_out/pmc_inf}
run() { timeout -s KILL 90 rocprofv3 --pmc $2 --output-format csv -d $OUT/$1 -o p -- python3 tools/bench_kernels.py --size-gb 1 --only inflate --reps 1 > $OUT/$1.log 2>&1; }
mkdir -p $OUT
run a "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES" || exit 1
run b "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_ANY" || exit 2
run c "FETCH_SIZE" || exit 3
run d "WRITE_SIZE GRBM_GUI_ACTIVE" || exit 4
run e "TCC_HIT_sum TCC_MISS_sum SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" || exit 5
