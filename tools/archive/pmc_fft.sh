#!/bin/bash
# Fourier-path kernel (k_fft_mfma) at cfg3 (or $CFG): bench line, kernel stats, then one rocprofv3 run per
# counter group (--kernel-trace only) and the summary (tools/pmc_summary_fft.py).
set -o pipefail
R=$GRAFT_REPO_ROOT
CFG=${CFG:-cfg3}
OUT=$R/gpurun_out/pmcfft_$CFG
mkdir -p $OUT
cd $R
timeout -k 10 200 python -u bench.py --config $CFG --steps 10 --warmup 2 --cpu-seconds 0 --no-extras > $OUT/bench.json 2> $OUT/bench.err || exit $?
cat $OUT/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- python3 $R/bench.py --config $CFG --steps 5 --warmup 1 --cpu-seconds 0 --no-parity --no-extras > $OUT/stats.log 2>&1 || exit $?
run() { name=$1; shift 1; timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -d $OUT/$name -o run --output-format csv -- python3 $R/bench.py --config $CFG --steps 2 --warmup 1 --cpu-seconds 0 --no-parity --no-extras > $OUT/$name.log 2>&1; }
run sq SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE || exit $?
run fetch FETCH_SIZE || exit $?
run write WRITE_SIZE || exit $?
run lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS || exit $?
run tcc TCC_HIT_sum TCC_MISS_sum || exit $?
run inst SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE || exit $?
cd $R
python3 tools/pmc_summary_fft.py $OUT ${KPAT:-k_fft_chunk} > $OUT/summary.txt 2>&1
cat $OUT/summary.txt
find $OUT/stats -name '*kernel_stats.csv' -exec head -6 {} \; | cut -c1-200
