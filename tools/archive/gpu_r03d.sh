#!/bin/bash
# k_fft_mfma segment stamps at cfg5 (diagnostic build) + the product kernel timing
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03d; mkdir -p $O
QCE_LIB=quantized_channel_estimation_amd/libqce_stamps.so timeout -k 10 200 python -u tools/fft_stamps.py cfg5 > $O/stamps_cfg5.txt 2>&1; rc=$?
cat $O/stamps_cfg5.txt; [ $rc -ne 0 ] && exit $rc
QCE_LIB=quantized_channel_estimation_amd/libqce_stamps.so timeout -k 10 200 python -u tools/fft_stamps.py cfg3 > $O/stamps_cfg3.txt 2>&1; rc=$?
cat $O/stamps_cfg3.txt; exit $rc
