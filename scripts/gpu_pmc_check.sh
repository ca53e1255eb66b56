# PMC passes on the full checker (4 GB)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/pmc_chk
mkdir -p $OUT
run() { timeout -s KILL 150 rocprofv3 --pmc $2 --output-format csv -d $OUT/$1 -o p -- python3 tools/bench_kernels.py --size-gb 4 --only check_full --reps 1 > $OUT/$1.log 2>&1; }
run a "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES" || exit 1
run b "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_ANY" || exit 2
run c "FETCH_SIZE" || exit 3
run d "WRITE_SIZE GRBM_GUI_ACTIVE" || exit 4
