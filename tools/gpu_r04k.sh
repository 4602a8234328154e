#!/bin/bash
# Round 4, build of the final kernels: PMC passes of cfg4 (k_est_all_f64, N = 128, with K=1 calibration), cfg3
# (k_fft_wreg, cycle passes at B = 1e6) and cfg5 (k_fft_chunk, cycle passes at B = 2e5), traffic JSONs stamped with
# the build, then one bench line per BASELINE config with that traffic.  Outputs under gpurun_out/r04k/ and pmc_*.
set -o pipefail
O=gpurun_out/r04k
mkdir -p $O
CFG=cfg4 KPAT=k_est_all_f64 CAL=1 TAG=cfg4 bash tools/pmc_kernel.sh | tail -12 || exit 1
CFG=cfg3 KPAT=k_fft_wreg BCYC=1000000 TAG=cfg3 bash tools/pmc_kernel.sh | tail -10 || exit 1
CFG=cfg5 KPAT=k_fft_chunk BCYC=200000 TAG=cfg5 bash tools/pmc_kernel.sh | tail -10 || exit 1
for C in cfg3 cfg4 cfg5; do cp gpurun_out/pmc_$C/traffic_$C.json profiles/traffic_$C.json || exit 1; done
for C in cfg1 cfg2 cfg3 cfg4 cfg5; do
  timeout -k 10 300 python -u bench.py --config $C --cpu-seconds 0 --no-extras > $O/$C.json 2> $O/$C.err || { tail -20 $O/$C.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$C.json'));r=d['roofline'];print('$C', d['value'], d['ms_per_step'], r.get('kernel_ms'), r['frac'], r.get('mfma_issue_frac'), r.get('fp64_frac'), r.get('traffic'), d['parity']['rel_fro'])"
done
