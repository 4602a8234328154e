#!/bin/bash
# Round-5 final bench lines of every configuration (this build), the cfg2 SNR sweep, and cfg4's PMC traffic.
set -o pipefail
mkdir -p gpurun_out/r05f
for c in cfg1 cfg2 cfg3 cfg4 cfg5; do
  timeout -k 10 300 python bench.py --config $c --no-extras > gpurun_out/r05f/${c}_bench.json 2> gpurun_out/r05f/${c}_bench.err || exit $?
done
for c in cfg3 cfg5; do
  timeout -k 10 200 python bench.py --config $c --mean --no-extras --cpu-seconds 0 > gpurun_out/r05f/${c}_mean_bench.json 2> gpurun_out/r05f/${c}_mean_bench.err || exit $?
done
timeout -k 10 200 python bench.py --config cfg2 --sweep --no-extras --cpu-seconds 0 > gpurun_out/r05f/cfg2_sweep.json 2> gpurun_out/r05f/cfg2_sweep.err || exit $?
CFG=cfg4 KPAT=k_est_all_f64 TAG=fcfg4 CAL=1 timeout -k 10 700 bash tools/pmc_kernel.sh > gpurun_out/pmc_fcfg4.log 2>&1 || exit $?
