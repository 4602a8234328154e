#!/bin/bash
# PMC passes of one estimate kernel (rocprofv3 --kernel-trace --pmc, one counter group per run, each under its own
# time limit), summarised by tools/pmc_report.py into <out>/summary.txt and profiles-ready traffic JSON.
#   CFG   bench config (metric, cfg3, cfg4, cfg5, ...)        KPAT  kernel-name pattern (k_est_all_f64, k_fft_wreg, ...)
#   BCYC  batch of the cycle-counter passes (default: the config's B; give the short Fourier kernels >= 0.3 ms
#         dispatches, MI355X_MICROARCH.md "DVFS give-back": GRBM_GUI_ACTIVE/8/time reads high below that)
#   CAL   1: K=1 calibration passes of FETCH/WRITE (dense kernels: y in + h out, tables negligible)
#   EXTRA extra bench.py arguments for every pass (e.g. --mean)
set -o pipefail
R=$GRAFT_REPO_ROOT
CFG=${CFG:-metric}
KPAT=${KPAT:-k_est_all_f64}
OUT=$R/gpurun_out/pmc_${TAG:-$CFG}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
BARGS=${BCYC:+--batch $BCYC}
run() { name=$1; shift; extra=$1; shift; timeout -k 10 -s KILL 150 rocprofv3 --kernel-trace --pmc "$@" -d $OUT/$name -o run --output-format csv -- python3 $R/bench.py --config $CFG --steps 2 --warmup 1 --cpu-seconds 0 --no-parity --no-extras $EXTRA $extra > $OUT/$name.log 2>&1; }
run sq "$BARGS" SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE || exit $?
run inst "$BARGS" SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE || exit $?
run lds "$BARGS" SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE || exit $?
run fetch "" FETCH_SIZE || exit $?
run write "" WRITE_SIZE || exit $?
run tcc "" TCC_HIT_sum TCC_MISS_sum || exit $?
run dram "" TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_DRAM_sum || exit $?
if [ "${CAL:-0}" = "1" ]; then
  run cfetch "--components 1" FETCH_SIZE || exit $?
  run cwrite "--components 1" WRITE_SIZE || exit $?
  run cdram "--components 1" TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_DRAM_sum || exit $?
fi
cd $R
BID=$(python3 -c "from quantized_channel_estimation_amd import _lib; print(_lib.build_id())")
TNAME=traffic_$CFG
case " $EXTRA " in *" --mean "*) TNAME=traffic_${CFG}_mean ;; esac
python3 tools/pmc_report.py $OUT "$KPAT" $CFG "$BID" $TNAME > $OUT/summary.txt 2>&1
cat $OUT/summary.txt
