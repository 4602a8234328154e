#!/bin/bash
# FP64 kernel round: its GPU tests, a metric bench line, rocprof kernel stats of the same command.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/f64; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_f64.py -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed|Error|assert" $O/pytest.log | tail -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 240 python -u bench.py --steps 10 --warmup 2 --cpu-seconds 0 > $O/bench.json 2> $O/bench.err || exit $?
cat $O/bench.json
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 -u bench.py --steps 10 --warmup 2 --cpu-seconds 0 --no-parity > $O/prof.log 2>&1 || exit $?
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/kernel_stats.csv
head -12 $O/kernel_stats.csv | cut -c1-200
