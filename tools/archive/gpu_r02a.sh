#!/bin/bash
# Round-2 GPU pass: full GPU suite, metric bench line (f64 headline + fast/drop-in side lines + CPU baseline),
# a 2-rank K-shard rehearsal on the one GPU (gloo), rocprof kernel stats of the metric command.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02a; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $O/pytest.log | tail -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 > $O/bench.json 2> $O/bench.err || exit $?
cat $O/bench.json
timeout -k 10 300 python -u bench.py --gpus 2 --backend gloo --collective ar --steps 3 --warmup 1 --batch 20000 > $O/bench_k2.json 2> $O/bench_k2.err || { tail -20 $O/bench_k2.err; exit 1; }
cat $O/bench_k2.json
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 -u bench.py --steps 10 --warmup 2 --cpu-seconds 0 --no-parity --no-extras > $O/prof.log 2>&1 || exit $?
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/kernel_stats.csv
head -8 $O/kernel_stats.csv | cut -c1-180
