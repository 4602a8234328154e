#!/bin/bash
# Round-6 final evidence for the current tree (outputs under gpurun_out/r06f/): the driver's bench command, its
# rocprofv3 kernel trace + stats (csv), the PMC passes of the headline kernel with K=1 calibration (traffic JSON stamped
# with this build's id, copied to profiles/), the bench line that picks that traffic up, every other configuration's
# bench line, and the emulated-rank K-shard steps (world 8 ranks 0 / 7 at K = 16, world 4 / 2, cfg4 K = 32).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06f
mkdir -p $O
cd $R
timeout -k 10 400 python -u bench.py > $O/metric_bench.json 2> $O/metric_bench.err || { tail -20 $O/metric_bench.err; exit 1; }
cat $O/metric_bench.json | cut -c1-300
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $O/prof.log 2> $O/prof.err || { tail -20 $O/prof.err; exit 1; }
cd $R
CFG=metric KPAT=k_est_all_f64 CAL=1 TAG=r06f_metric bash tools/pmc_kernel.sh > $O/pmc_metric.txt 2>&1 || { tail -20 $O/pmc_metric.txt; exit 1; }
cp gpurun_out/pmc_r06f_metric/traffic_metric.json profiles/traffic_metric.json
cp gpurun_out/pmc_r06f_metric/traffic_metric.json $O/traffic_metric.json
timeout -k 10 400 python -u bench.py --cpu-seconds 0 --no-extras > $O/metric_bench_traffic.json 2> $O/metric_bench_traffic.err || exit 1
for c in cfg1 cfg2 cfg3 cfg4 cfg5; do
  timeout -k 10 300 python bench.py --config $c --no-extras --cpu-seconds 0 > $O/${c}_bench.json 2> $O/${c}_bench.err || exit 1
done
timeout -k 10 200 python tools/kshard_native_step.py --K 16 --steps 40 --emulate-world 8:0 > $O/rank16_r0.json 2> $O/rank16_r0.err || exit 1
timeout -k 10 200 python tools/kshard_native_step.py --K 16 --steps 40 --emulate-world 8:7 > $O/rank16_r7.json 2> $O/rank16_r7.err || exit 1
timeout -k 10 200 python tools/kshard_native_step.py --K 32 --steps 30 --emulate-world 4:0 > $O/rank32_w4.json 2> $O/rank32_w4.err || exit 1
timeout -k 10 200 python tools/kshard_native_step.py --K 64 --steps 20 --emulate-world 2:0 > $O/rank64_w2.json 2> $O/rank64_w2.err || exit 1
timeout -k 10 200 python tools/kshard_native_step.py --K 32 --N 128 --B 50000 --steps 20 --emulate-world 8:0 > $O/cfg4_rank32.json 2> $O/cfg4_rank32.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_rank16 -o run --output-format csv -- python3 $R/tools/kshard_native_step.py --K 16 --steps 40 --emulate-world 8:0 --no-parity > $O/prof_rank16.log 2> $O/prof_rank16.err || { tail -20 $O/prof_rank16.err; exit 1; }
cd $R
echo done
