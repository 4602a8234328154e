#!/bin/bash
# Round 4: A/B of the FP64 headline kernel's launch shape (8-wave workgroup vs two 4-wave workgroups per CU), each
# with its parity line, then the FP64 tests under the new shape.
set -o pipefail
mkdir -p gpurun_out/r04b
for V in 8:0 42:0 8:1 42:1 8:0 42:0 8:1 42:1; do
  W=${V%:*}; P=${V#*:}
  QCE_F64_WAVES=$W QCE_F64_PIPE=$P timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --cpu-seconds 0 --no-extras > gpurun_out/r04b/bench_w${W}p$P.json 2> gpurun_out/r04b/bench_w${W}p$P.err || { tail -20 gpurun_out/r04b/bench_w${W}p$P.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r04b/bench_w${W}p$P.json'));r=d['roofline'];print('W=$W P=$P', d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], r.get('mfma_issue_frac'), d['parity']['rel_fro'])"
done
QCE_F64_WAVES=42 QCE_F64_PIPE=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_f64.py tests/test_gpu_fullbatch.py tests/test_gpu_argmax_metric.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04b/pytest42.log 2>&1 || { tail -30 gpurun_out/r04b/pytest42.log; exit 1; }
tail -2 gpurun_out/r04b/pytest42.log
