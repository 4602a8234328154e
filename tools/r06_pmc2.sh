#!/bin/bash
# Round-6 final PMC traffic of this build: the Fourier kernels of cfg3 / cfg5, zero-mean and with means.
set -o pipefail
CFG=cfg3 KPAT=k_fft_wreg TAG=r6cfg3 BCYC=400000 timeout -k 10 400 bash tools/pmc_kernel.sh > gpurun_out/pmc_r6cfg3.log 2>&1 || exit $?
CFG=cfg5 KPAT=k_fft_chunk TAG=r6cfg5 timeout -k 10 400 bash tools/pmc_kernel.sh > gpurun_out/pmc_r6cfg5.log 2>&1 || exit $?
CFG=cfg3 KPAT=k_fft_wreg TAG=r6cfg3mean EXTRA=--mean BCYC=200000 timeout -k 10 400 bash tools/pmc_kernel.sh > gpurun_out/pmc_r6cfg3mean.log 2>&1 || exit $?
CFG=cfg5 KPAT=k_fft_chunk_hm TAG=r6cfg5mean EXTRA=--mean timeout -k 10 400 bash tools/pmc_kernel.sh > gpurun_out/pmc_r6cfg5mean.log 2>&1 || exit $?
