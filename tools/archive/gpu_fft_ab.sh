#!/bin/bash
# Fourier-path parity tests, then cfg3 / cfg5 bench lines for each QCE_FFT_SCHED value in $VARS.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/fab; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "${SEL:-fourier}" > $O/pytest.log 2>&1
rc=$?; grep -E "passed|failed|Error|assert" $O/pytest.log | tail -5; [ $rc -ne 0 ] && exit $rc
for v in ${VARS:-1 0}; do
  for c in ${CFGS:-cfg3}; do
    QCE_FFT_SCHED=$v timeout -k 10 200 python -u bench.py --config $c --steps 20 --warmup 3 --cpu-seconds 0 --no-extras > $O/$c.$v.json 2> $O/$c.$v.err || exit $?
    python -c "import json;d=json.load(open('$O/$c.$v.json'));print('$c sched=$v',d['value'],d['roofline']['kernel_ms'],d['roofline']['frac'],d['parity']['rel_fro'])"
  done
done
if [ -n "$METRIC" ]; then
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --cpu-seconds 0 > $O/metric.json 2> $O/metric.err || exit $?
  python -c "import json;d=json.load(open('$O/metric.json'));print('metric',d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],'dropin',d.get('dropin'))"
fi
