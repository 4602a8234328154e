#!/bin/bash
# Round 6 measurements of this build: the metric bench line + rocprofv3 stats of the same command, the drop-in side
# line, every config's line, the cfg2 sweep, and the emulated world-8 rank steps (metric K=16, cfg4 K=32).
# Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
R=$PWD
O=$R/gpurun_out/r06m
mkdir -p $O
timeout -k 10 300 python bench.py > $O/metric_bench.json 2> $O/metric_bench.err || exit $?
for c in cfg1 cfg2 cfg3 cfg4 cfg5; do
  timeout -k 10 300 python bench.py --config $c --no-extras > $O/${c}_bench.json 2> $O/${c}_bench.err || exit $?
done
for c in metric cfg2 cfg3 cfg4 cfg5; do
  timeout -k 10 200 python bench.py --config $c --mean --no-extras --cpu-seconds 0 > $O/${c}_mean_bench.json 2> $O/${c}_mean_bench.err || exit $?
done
timeout -k 10 200 python bench.py --config cfg2 --sweep --no-extras --cpu-seconds 0 > $O/cfg2_sweep.json 2> $O/cfg2_sweep.err || exit $?
timeout -k 10 200 python bench.py --dropin --no-extras --cpu-seconds 0 --steps 5 > $O/dropin_bench.json 2> $O/dropin.err || exit $?
for ew in 8:0 8:7 4:0 2:0; do
  timeout -k 10 200 python tools/kshard_native_step.py --K $((128 / ${ew%%:*})) --steps 20 --emulate-world $ew > $O/rank_metric_${ew/:/_}.json 2> $O/rank_metric_${ew/:/_}.err || exit $?
done
timeout -k 10 300 python tools/kshard_native_step.py --K 32 --N 128 --B 50000 --steps 10 --emulate-world 8:0 > $O/rank_cfg4_8_0.json 2> $O/rank_cfg4.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_metric -o run --output-format csv -- python3 $R/bench.py > $O/metric_bench_prof.json 2> $O/metric_bench_prof.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_cfg4 -o run --output-format csv -- python3 $R/bench.py --config cfg4 --no-extras --cpu-seconds 0 > $O/cfg4_prof.json 2> $O/cfg4_prof.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_rank16 -o run --output-format csv -- python3 $R/tools/kshard_native_step.py --K 16 --steps 20 --emulate-world 8:0 > $O/rank16_prof.json 2> $O/rank16_prof.err || exit $?
echo done
