#!/bin/bash
# Round 4: A/B of the FP64 kernel's LDS prefetch distance (QCE_F64_E = 2 default, 3, 4; libqce_e3/e4.so via QCE_LIB)
# at the metric config and cfg4, two rounds on one box.
set -o pipefail
mkdir -p gpurun_out/r04g
L=quantized_channel_estimation_amd
for r in 1 2; do for V in libqce_e6 libqce_e8 libqce_e10 libqce_e12; do for C in metric; do
  QCE_LIB=$L/$V.so timeout -k 10 300 python -u bench.py --config $C --steps 8 --warmup 2 --cpu-seconds 0 --no-extras > gpurun_out/r04g/${V}_$C.json 2> gpurun_out/r04g/err.txt || { tail -20 gpurun_out/r04g/err.txt; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r04g/${V}_$C.json'));r=d['roofline'];print('$V $C', d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], r.get('mfma_issue_frac'), d['parity']['rel_fro'])"
done; done; done
