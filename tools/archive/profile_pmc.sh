#!/bin/bash
# PMC passes for the fused estimate kernel (run on the GPU box from the repo root).
# Each counter group is its own rocprofv3 run with --kernel-trace only (no sys/runtime traces).
set -e
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
BENCH="python $R/bench.py --steps 3 --warmup 1 --cpu-seconds 0 --no-parity"
rocprofv3 -L > $OUT/counters.txt 2>&1 || true
run() { name=$1; shift; timeout -k 10 -s KILL 150 rocprofv3 --kernel-trace --pmc "$@" -d $OUT/$name -o run --output-format csv -- $BENCH > $OUT/$name.log 2>&1; }
run fetch FETCH_SIZE
run write WRITE_SIZE
run sq SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
run lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS
run tcc TCC_HIT_sum TCC_MISS_sum
echo done
