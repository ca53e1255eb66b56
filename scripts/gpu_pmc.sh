# PMC passes on the bench workload (10 GB): HBM traffic (FETCH_SIZE, WRITE_SIZE), SQ instruction counts and SQ
# stall/wait cycles, one counter group per pass; summary → gpurun_out/pmc/traffic.json (copy into profiles/<round>/)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/pmc
mkdir -p $OUT
ONLY=${ONLY:-inflate,check_full,check_eager}
run() { timeout -s KILL 240 rocprofv3 --pmc $2 --output-format csv -d $OUT/$1 -o p -- python3 tools/bench_kernels.py --size-gb 10 --only $ONLY --reps 1 > $OUT/$1.log 2>&1; }
run f "FETCH_SIZE" || exit 2
run w "WRITE_SIZE" || exit 3
run sq1 "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM" || exit 4
run sq2 "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM" || exit 5
run sq3 "GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES" || exit 7
python3 tools/traffic_pmc.py $OUT/traffic.json $OUT/f $OUT/w --sq-dir $OUT/sq1 --sq-dir $OUT/sq2 --sq-dir $OUT/sq3 > $OUT/summary.log 2>&1 || exit 6
