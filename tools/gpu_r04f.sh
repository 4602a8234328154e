#!/bin/bash
# Round 4: segment stamps of k_est_all_f64 (diagnostic build) at the metric config and cfg4, then the Fourier
# kernels' PMC passes with a reliable cycle base (cfg3 k_fft_wreg at B = 1e6 for the cycle passes, cfg5 k_fft_chunk
# at B = 2e5), traffic at the configs' own B.
set -o pipefail
mkdir -p gpurun_out/r04f
for C in metric cfg4; do
  QCE_LIB=quantized_channel_estimation_amd/libqce_stamps.so timeout -k 10 300 python -u tools/f64_stamps.py $C > gpurun_out/r04f/stamps_$C.txt 2>&1 || { tail -20 gpurun_out/r04f/stamps_$C.txt; exit 1; }
  cat gpurun_out/r04f/stamps_$C.txt
done
CFG=cfg3 KPAT=k_fft_wreg BCYC=1000000 TAG=cfg3 bash tools/pmc_kernel.sh || exit 1
CFG=cfg5 KPAT=k_fft_chunk BCYC=200000 TAG=cfg5 bash tools/pmc_kernel.sh || exit 1
