#!/bin/bash
# Round-5 final PMC traffic of this build: the metric kernel (with the K=1 calibration passes) and the Fourier
# kernels of cfg3 / cfg5, zero-mean and with means (tools/pmc_kernel.sh, one counter group per pass, each under its
# own time limit; summaries + traffic_<config>[_mean].json under gpurun_out/pmc_<tag>/).
set -o pipefail
CFG=metric KPAT=k_est_all_f64g TAG=fmetric CAL=1 timeout -k 10 600 bash tools/pmc_kernel.sh > gpurun_out/pmc_fmetric.log 2>&1 || exit $?
CFG=cfg3 KPAT=k_fft_wreg TAG=fcfg3 BCYC=400000 timeout -k 10 500 bash tools/pmc_kernel.sh > gpurun_out/pmc_fcfg3.log 2>&1 || exit $?
CFG=cfg5 KPAT=k_fft_chunk TAG=fcfg5 timeout -k 10 500 bash tools/pmc_kernel.sh > gpurun_out/pmc_fcfg5.log 2>&1 || exit $?
CFG=cfg3 KPAT=k_fft_wreg TAG=fcfg3mean EXTRA=--mean BCYC=200000 timeout -k 10 500 bash tools/pmc_kernel.sh > gpurun_out/pmc_fcfg3mean.log 2>&1 || exit $?
CFG=cfg5 KPAT=k_fft_chunk_hm TAG=fcfg5mean EXTRA=--mean timeout -k 10 500 bash tools/pmc_kernel.sh > gpurun_out/pmc_fcfg5mean.log 2>&1 || exit $?
