#!/bin/bash
# Quick perf check: f64 tests (fast subset), metric + cfg4 lines, stamp breakdown.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/quick; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_f64.py -x -q --timeout 180 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --cpu-seconds 0 --no-extras > $O/bench.json 2> $O/bench.err || exit $?
python3 -c "import json;d=json.load(open('$O/bench.json'));r=d['roofline'];print('metric',d['value'],d['ms_per_step'],r['kernel_ms'],r['frac'],r['mfma_issue_frac'],d['parity']['rel_fro'])"
timeout -k 10 300 python -u bench.py --config cfg4 --steps 3 --warmup 1 --cpu-seconds 0 > $O/bench4.json 2> $O/bench4.err || exit $?
python3 -c "import json;d=json.load(open('$O/bench4.json'));r=d['roofline'];print('cfg4',d['value'],d['ms_per_step'],r['kernel_ms'],r['frac'],r['mfma_issue_frac'],d['parity']['rel_fro'])"
QCE_LIB=quantized_channel_estimation_amd/libqce_stamps.so timeout -k 10 300 python3 -u tools/f64_stamps.py
