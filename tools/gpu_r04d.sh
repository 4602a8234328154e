#!/bin/bash
# Round 4: deeper LDS ring (>= 96 blocks of prefetch lead) for the one-wave-per-SIMD FP64 shapes (padded 128): cfg4
# bench lines, the FP64 tests at those shapes, the metric line as a regression check.
set -o pipefail
mkdir -p gpurun_out/r04d
for i in 1 2; do
timeout -k 10 300 python -u bench.py --config cfg4 --steps 10 --warmup 2 --cpu-seconds 0 > gpurun_out/r04d/cfg4_$i.json 2> gpurun_out/r04d/cfg4.err || { tail -20 gpurun_out/r04d/cfg4.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r04d/cfg4_$i.json'));r=d['roofline'];print('cfg4', d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], r.get('mfma_issue_frac'), d['parity']['rel_fro'])"
done
timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --cpu-seconds 0 --no-extras > gpurun_out/r04d/metric.json 2> gpurun_out/r04d/metric.err || { tail -20 gpurun_out/r04d/metric.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r04d/metric.json'));r=d['roofline'];print('metric', d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], r.get('mfma_issue_frac'), d['parity']['rel_fro'])"
timeout -k 10 500 python -u -m pytest tests/test_gpu_f64.py tests/test_gpu_fullbatch.py tests/test_gpu_configs.py -x -q --timeout 170 --timeout-method thread > gpurun_out/r04d/pytest.log 2>&1 || { tail -40 gpurun_out/r04d/pytest.log; exit 1; }
tail -2 gpurun_out/r04d/pytest.log
