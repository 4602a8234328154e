#!/bin/bash
# k_fft_chunk buffer loads / unrolled filter / table exp: Fourier tests, cfg5 bench A/B vs the bin-split kernel
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03k; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -k "fourier or cfg5 or fft or cfg3 or fullbatch" > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; grep -E "FAILED|Error" $O/pytest.log | head -10
[ $rc -ne 0 ] && exit $rc
for v in 1 0 1; do
  QCE_FFT_CHUNK=$v timeout -k 10 200 python -u bench.py --config cfg5 --steps 10 --warmup 2 --cpu-seconds 0 > $O/cfg5_$v.json 2> $O/cfg5_$v.err || exit $?
  python -c "import json;d=json.load(open('$O/cfg5_$v.json'));print('cfg5 chunk=$v',d['value'],d['roofline']['kernel_ms'],d['roofline']['frac'],d['parity']['rel_fro'])"
done
