#!/bin/bash
# Round-6 final PMC traffic of this build: the metric kernel (k_est_all_f64g, with the K=1 calibration passes) and
# cfg4's k_est_all_f64h (tools/pmc_kernel.sh: one counter group per pass, each under its own time limit).
set -o pipefail
CFG=metric KPAT=k_est_all_f64g TAG=r6metric CAL=1 timeout -k 10 560 bash tools/pmc_kernel.sh > gpurun_out/pmc_r6metric.log 2>&1 || exit $?
CFG=cfg4 KPAT=k_est_all_f64h TAG=r6cfg4 CAL=1 timeout -k 10 560 bash tools/pmc_kernel.sh > gpurun_out/pmc_r6cfg4.log 2>&1 || exit $?
