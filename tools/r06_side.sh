#!/bin/bash
# Round 6 final build: side lines -- dense with means at the metric config (the reference's fit default), the drop-in
# numpy call, the cfg2 SNR sweep.
set -o pipefail
R=$PWD
O=$R/gpurun_out/r06side
mkdir -p $O
timeout -k 10 300 python bench.py --mean --no-extras --cpu-seconds 0 > $O/metric_mean_bench.json 2> $O/metric_mean_bench.err || exit 1
timeout -k 10 300 python bench.py --dropin --no-extras --cpu-seconds 0 > $O/dropin_bench.json 2> $O/dropin_bench.err || exit 1
timeout -k 10 300 python bench.py --config cfg2 --sweep --no-extras --cpu-seconds 0 > $O/sweep_cfg2.json 2> $O/sweep_cfg2.err || exit 1
echo done
