#!/bin/bash
# current k_fft_chunk<256> at cfg5: segment stamps (diagnostic build) and PMC passes
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03p; mkdir -p $O
QCE_LIB=quantized_channel_estimation_amd/libqce_stamps.so timeout -k 10 200 python -u tools/fft_stamps.py cfg5 > $O/stamps_cfg5.txt 2>&1 || { cat $O/stamps_cfg5.txt; exit 1; }
cat $O/stamps_cfg5.txt
QCE_LIB=quantized_channel_estimation_amd/libqce_stamps.so timeout -k 10 200 python -u tools/fft_stamps.py cfg3 > $O/stamps_cfg3.txt 2>&1 || { cat $O/stamps_cfg3.txt; exit 1; }
cat $O/stamps_cfg3.txt
CFG=cfg5 KPAT=k_fft_chunk timeout -k 10 600 bash tools/pmc_fft.sh > $O/pmc5.log 2>&1 || exit $?
tail -8 $O/pmc5.log
