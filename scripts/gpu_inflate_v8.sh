# decode select tree as v_cndmask: parity, 10 GB timing, PMC instruction mix of the inflate kernels (1 GB)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_inflate_streams.py tests/test_gpu_parity.py -x -q -m gpu -k "inflate or stream" --timeout 120 --timeout-method thread > gpurun_out/pytest_inflate.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_kernels.py --size-gb 10 --only inflate --reps 2 > gpurun_out/kern10.log 2>&1 || exit 2
OUT=gpurun_out/pmc_inf8
run() { timeout -s KILL 90 rocprofv3 --pmc $2 --output-format csv -d $OUT/$1 -o p -- python3 tools/bench_kernels.py --size-gb 1 --only inflate --reps 1 > $OUT/$1.log 2>&1; }
mkdir -p $OUT
run a "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES" || exit 3
run b "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_ANY" || exit 4
