#!/bin/bash
# Fourier-path state: cfg3 / cfg5 bench lines + kernel stats, then k_fft_mfma / k_fft_wave segment stamps (diagnostic build)
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03e; mkdir -p $O
for c in cfg3 cfg5; do
  timeout -k 10 200 python -u bench.py --config $c --steps 10 --warmup 2 --cpu-seconds 0 > $O/$c.json 2> $O/$c.err || exit $?
  python -c "import json;d=json.load(open('$O/$c.json'));print('$c',d['value'],d['roofline']['kernel_ms'],d['roofline']['frac'],d['parity'])"
done
QCE_LIB=quantized_channel_estimation_amd/libqce_stamps.so timeout -k 10 200 python -u tools/fft_stamps.py cfg5 > $O/stamps_cfg5.txt 2>&1 || { cat $O/stamps_cfg5.txt; exit 1; }
cat $O/stamps_cfg5.txt
QCE_LIB=quantized_channel_estimation_amd/libqce_stamps.so timeout -k 10 200 python -u tools/fft_stamps.py cfg3 > $O/stamps_cfg3.txt 2>&1 || { cat $O/stamps_cfg3.txt; exit 1; }
cat $O/stamps_cfg3.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/stats5 -o run --output-format csv -- python3 $R/bench.py --config cfg5 --steps 5 --warmup 1 --cpu-seconds 0 --no-parity --no-extras > $O/stats5.log 2>&1 || exit $?
find $O/stats5 -name '*kernel_stats.csv' -exec head -4 {} \; | cut -c1-200
