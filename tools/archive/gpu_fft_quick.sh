#!/bin/bash
# Fourier-path parity tests then short cfg3 / cfg5 bench lines (no CPU baseline).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/fq; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "${SEL:-fourier}" > $O/pytest.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed|Error|assert" $O/pytest.log | tail -30; [ $rc -ne 0 ] && exit $rc
for c in cfg3 cfg5; do
  timeout -k 10 200 python -u bench.py --config $c --steps 10 --warmup 2 --cpu-seconds 0 > $O/$c.json 2> $O/$c.err || exit $?
  python -c "import json;d=json.load(open('$O/$c.json'));print('$c',d['value'],d['roofline']['kernel_ms'],d['roofline']['frac'],d['parity'])"
done
