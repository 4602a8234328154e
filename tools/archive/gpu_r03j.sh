#!/bin/bash
# round-3 library: cfg1 / cfg2 / cfg4 bench lines, then cfg3 PMC passes for k_fft_wreg
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03j; mkdir -p $O
for c in cfg1 cfg2 cfg4; do
  timeout -k 10 300 python -u bench.py --config $c --steps 10 --warmup 2 --cpu-seconds 0 > $O/$c.json 2> $O/$c.err || exit $?
  python -c "import json;d=json.load(open('$O/$c.json'));r=d['roofline'];print('$c',d['value'],d['ms_per_step'],r['kernel_ms'],r['frac'],r.get('mfma_issue_frac'),d['parity']['rel_fro'])"
done
CFG=cfg3 KPAT=k_fft_wreg timeout -k 10 600 bash tools/pmc_fft.sh > $O/pmc3.log 2>&1 || exit $?
tail -12 $O/pmc3.log
