#!/bin/bash
# A/B of the FP64 kernel's workgroup shape at the metric config (4 waves x 2 column tiles vs 8 x 1), tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/ab; mkdir -p $O
for wv in 4 8; do
  QCE_F64_WAVES=$wv timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --cpu-seconds 0 --no-extras > $O/bench_$wv.json 2> $O/bench_$wv.err || exit $?
  python3 -c "import json;d=json.load(open('$O/bench_$wv.json'));r=d['roofline'];print('waves $wv',d['value'],d['ms_per_step'],r['kernel_ms'],r['frac'],r['mfma_issue_frac'],d['parity']['rel_fro'])"
done
timeout -k 10 300 python -u bench.py --config cfg4 --steps 3 --warmup 1 --cpu-seconds 0 > $O/bench4.json 2> $O/bench4.err || exit $?
python3 -c "import json;d=json.load(open('$O/bench4.json'));r=d['roofline'];print('cfg4',d['value'],d['ms_per_step'],r['kernel_ms'],r['frac'],r['mfma_issue_frac'],d['parity']['rel_fro'])"
for wv in 4 8; do
QCE_F64_WAVES=$wv timeout -k 10 300 python -u -m pytest tests/test_gpu_f64.py -x -q --timeout 180 --timeout-method thread > $O/pytest$wv.log 2>&1; rc=$?; tail -1 $O/pytest$wv.log; [ $rc -ne 0 ] && exit $rc
done
QCE_F64_WAVES=8 QCE_LIB=quantized_channel_estimation_amd/libqce_stamps.so timeout -k 10 300 python3 -u tools/f64_stamps.py
