#!/bin/bash
# k_fft_wreg (N = 64) + k_fft_chunk: Fourier tests, cfg3 A/B (QCE_FFT_CHUNK=1 new kernels / 0 previous), cfg5, stamps
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03h; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -k "fourier or cfg5 or fft or cfg3" > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; grep -E "FAILED|Error" $O/pytest.log | head -10
[ $rc -ne 0 ] && exit $rc
for v in 1 0; do
  QCE_FFT_CHUNK=$v timeout -k 10 200 python -u bench.py --config cfg3 --steps 10 --warmup 2 --cpu-seconds 0 > $O/cfg3_$v.json 2> $O/cfg3_$v.err || exit $?
  python -c "import json;d=json.load(open('$O/cfg3_$v.json'));print('cfg3 chunk=$v',d['value'],d['roofline']['kernel_ms'],d['roofline']['frac'],d['parity']['rel_fro'])"
done
timeout -k 10 200 python -u bench.py --config cfg5 --steps 10 --warmup 2 --cpu-seconds 0 > $O/cfg5.json 2> $O/cfg5.err || exit $?
python -c "import json;d=json.load(open('$O/cfg5.json'));print('cfg5',d['value'],d['roofline']['kernel_ms'],d['roofline']['frac'],d['parity']['rel_fro'])"
QCE_LIB=quantized_channel_estimation_amd/libqce_stamps.so timeout -k 10 200 python -u tools/fft_stamps.py cfg3 > $O/stamps_cfg3.txt 2>&1 || { cat $O/stamps_cfg3.txt; exit 1; }
cat $O/stamps_cfg3.txt
