#!/bin/bash
# Round 4, final kernels: LDS prefetch distance of k_est_all_f64 at the metric config (E = 8 default, libqce_e6 /
# libqce_e10 via QCE_LIB; padded 128 keeps its E = 4), two rounds.  Data for the next round; the default is unchanged.
set -o pipefail
O=gpurun_out/r04r
mkdir -p $O
L=quantized_channel_estimation_amd
for r in 1 2; do for V in libqce libqce_e6 libqce_e10; do
  QCE_LIB=$L/$V.so timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --cpu-seconds 0 --no-extras > $O/$V.json 2> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$V.json'));r=d['roofline'];print('$V metric', d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], r.get('mfma_issue_frac'), d['parity']['rel_fro'])" | tee -a $O/ab.txt
done; done
