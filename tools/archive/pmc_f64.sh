#!/bin/bash
# PMC passes of the FP64 fused kernel at the metric configuration (one rocprofv3 run per counter group,
# --kernel-trace only), plus K=1 calibration passes for FETCH_SIZE / WRITE_SIZE (y read + h write only).
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc64
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
run() { name=$1; comps=$2; shift 2; timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -d $OUT/$name -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --cpu-seconds 0 --no-parity --no-extras --components $comps > $OUT/$name.log 2>&1; }
run sq 128 SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE || exit $?
run fetch 128 FETCH_SIZE || exit $?
run write 128 WRITE_SIZE || exit $?
run lds 128 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS || exit $?
run tcc 128 TCC_HIT_sum TCC_MISS_sum || exit $?
run cfetch 1 FETCH_SIZE || exit $?
run cwrite 1 WRITE_SIZE || exit $?
cd $R
python3 tools/pmc_summary_f64.py gpurun_out/pmc64 k_est_all_f64 gpurun_out/pmc64/traffic_f64.json > gpurun_out/pmc64/summary.txt 2>&1
cat gpurun_out/pmc64/summary.txt
