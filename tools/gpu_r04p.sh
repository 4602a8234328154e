#!/bin/bash
# Round 4, final kernels: segment stamps of k_est_all_f64 (diagnostic -DQCE_STAMPS build) at the metric config and
# cfg4 (wave pairs).  Outputs under gpurun_out/r04p/.
set -o pipefail
O=gpurun_out/r04p
mkdir -p $O
for C in metric cfg4; do
  QCE_LIB=quantized_channel_estimation_amd/libqce_stamps.so timeout -k 10 300 python -u tools/f64_stamps.py $C > $O/stamps_$C.txt 2>&1 || { tail -20 $O/stamps_$C.txt; exit 1; }
  grep -v amdgpu.ids $O/stamps_$C.txt
done
