#!/bin/bash
# prepare A/B (k_zgemm VALU vs k_zgemm_mfma) on the metric and cfg4 benches, prepare kernel stats, then cfg3 PMC
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03j; mkdir -p $O
for v in mfma valu; do
  for c in metric cfg4; do
    QCE_ZGEMM=$v timeout -k 10 300 python -u bench.py --config $c --steps 10 --warmup 2 --cpu-seconds 0 --no-extras > $O/${c}_$v.json 2> $O/${c}_$v.err || exit $?
    python -c "import json;d=json.load(open('$O/${c}_$v.json'));r=d['roofline'];print('$c zgemm=$v',d['value'],d['ms_per_step'],r['kernel_ms'],round(d['ms_per_step']-r['kernel_ms'],4),d['parity']['rel_fro'])"
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prep -o run --output-format csv -- python3 $R/bench.py --config metric --steps 5 --warmup 1 --cpu-seconds 0 --no-parity --no-extras > $O/prep.log 2>&1 || exit $?
cd $R
python3 tools/trace_summary.py $(find $O/prep -name '*kernel_trace.csv' | head -1) "" > $O/prep_trace_summary.txt
cat $O/prep_trace_summary.txt
CFG=cfg3 KPAT=k_fft_wreg timeout -k 10 600 bash tools/pmc_fft.sh > $O/pmc3.log 2>&1 || exit $?
tail -12 $O/pmc3.log
