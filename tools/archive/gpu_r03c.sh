#!/bin/bash
# Fourier-path tests (all of them), the dense-256 config tests, cfg3 / cfg5 bench lines and cfg5 kernel stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03c; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread -k "fourier or cfg5 or dense_padded or fft or kshard" > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; grep -E "FAILED|Error" $O/pytest.log | head -10
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
for c in cfg3 cfg5; do
  timeout -k 10 200 python -u bench.py --config $c --steps 10 --warmup 2 --cpu-seconds 0 > $O/$c.json 2> $O/$c.err || exit $?
  python -c "import json;d=json.load(open('$O/$c.json'));print('$c',d['value'],d['roofline']['kernel_ms'],d['roofline']['frac'],d['parity'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/stats5 -o run --output-format csv -- python3 $R/bench.py --config cfg5 --steps 5 --warmup 1 --cpu-seconds 0 --no-parity --no-extras > $O/stats5.log 2>&1 || exit $?
find $O/stats5 -name '*kernel_stats.csv' -exec head -4 {} \; | cut -c1-200
exit $rc
