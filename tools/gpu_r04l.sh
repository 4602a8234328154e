#!/bin/bash
# Round 4: A/B of the ring barrier without the LDS-read drain (libqce) vs with it (libqce_drain, QCE_F64_BND_DRAIN=1),
# both with the permlane group sum; metric and cfg4, two rounds; then the FP64 parity tests on libqce.
set -o pipefail
O=gpurun_out/r04l
mkdir -p $O
L=quantized_channel_estimation_amd
for r in 1 2; do for V in libqce libqce_drain; do for C in metric cfg4; do
  QCE_LIB=$L/$V.so timeout -k 10 300 python -u bench.py --config $C --steps 10 --warmup 2 --cpu-seconds 0 --no-extras > $O/${V}_$C.json 2> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
  python3 -c "import json;d=json.load(open('$O/${V}_$C.json'));r=d['roofline'];print('$V $C', d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], r.get('mfma_issue_frac'), d['parity']['rel_fro'])" | tee -a $O/ab.txt
done; done; done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullbatch.py tests/test_gpu_configs.py tests/test_gpu_kshard_native.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
