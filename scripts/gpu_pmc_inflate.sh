# PMC passes on the inflate kernel (scan+inflate microbenchmark)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
run() { timeout -s KILL 90 rocprofv3 --pmc $2 --output-format csv -d gpurun_out/pmc_inf/$1 -o p -- python3 tools/bench_kernels.py --size-gb 1 --only inflate --reps 1 > gpurun_out/pmc_inf/$1.log 2>&1; }
mkdir -p gpurun_out/pmc_inf
run a "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES" || exit 1
run b "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_ANY" || exit 2
run c "FETCH_SIZE" || exit 3
run d "WRITE_SIZE GRBM_GUI_ACTIVE" || exit 4
run e "TA_BUSY_avr TCC_HIT_sum TCC_MISS_sum" || exit 5
