#!/bin/bash
# k_fft_chunk: Fourier tests, cfg5 bench (chunk vs bin-split A/B on the same box), cfg5 kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03f; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -k "fourier or cfg5 or fft" > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; grep -E "FAILED|Error" $O/pytest.log | head -10
[ $rc -ne 0 ] && exit $rc
for v in 1 0; do
  QCE_FFT_CHUNK=$v timeout -k 10 200 python -u bench.py --config cfg5 --steps 10 --warmup 2 --cpu-seconds 0 > $O/cfg5_$v.json 2> $O/cfg5_$v.err || exit $?
  python -c "import json;d=json.load(open('$O/cfg5_$v.json'));print('cfg5 chunk=$v',d['value'],d['roofline']['kernel_ms'],d['roofline']['frac'],d['parity']['rel_fro'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/stats5 -o run --output-format csv -- python3 $R/bench.py --config cfg5 --steps 5 --warmup 1 --cpu-seconds 0 --no-parity --no-extras > $O/stats5.log 2>&1 || exit $?
find $O/stats5 -name '*kernel_stats.csv' -exec head -4 {} \; | cut -c1-150
cd $R
QCE_LIB=quantized_channel_estimation_amd/libqce_stamps.so timeout -k 10 200 python -u tools/fft_stamps.py cfg5 > $O/stamps_cfg5.txt 2>&1 || { cat $O/stamps_cfg5.txt; exit 1; }
cat $O/stamps_cfg5.txt
