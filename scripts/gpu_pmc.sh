# PMC passes (one counter group per rocprofv3 run) on the checker-only microbenchmark
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
LIB=${1:-build}
run() { SBAM_LIB=spark-bam_amd/$LIB/libsbam.so timeout -s KILL 90 rocprofv3 --pmc $2 --output-format csv -d gpurun_out/pmc_$LIB/$1 -o p -- python3 tools/bench_kernels.py --size-gb 1 --only check_full --reps 1 > gpurun_out/pmc_$LIB/$1.log 2>&1; }
mkdir -p gpurun_out/pmc_$LIB
run a "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES" || exit 1
run b "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_ANY" || exit 2
run c "FETCH_SIZE" || exit 3
run d "WRITE_SIZE GRBM_GUI_ACTIVE" || exit 4
