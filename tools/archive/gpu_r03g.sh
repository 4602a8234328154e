#!/bin/bash
# k_fft_chunk de-phase experiment at cfg5: delay one parity class of the first-round workgroups
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03g; mkdir -p $O
for d in "0,0" "4,7" "0,0" "4,7" "8,7" "12,7" "4,6" "8,6" "4,9" "2,7"; do
  QCE_FFT_DEPHASE=$d timeout -k 10 200 python -u bench.py --config cfg5 --steps 10 --warmup 2 --cpu-seconds 0 --no-parity > $O/cfg5_$d.json 2> $O/cfg5_$d.err || exit $?
  python -c "import json;d=json.load(open('$O/cfg5_$d.json'));print('dephase $d',d['value'],d['roofline']['kernel_ms'])"
done
