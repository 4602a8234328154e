#!/bin/bash
# Observation-row GPU checks: parity tests, kernel throughput, rocprofv3 kernel stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/obs; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_observe.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed|Error|assert" $O/pytest.log | tail -30; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/bench_observe.py > $O/bench.jsonl 2> $O/bench.err || exit $?
cat $O/bench.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run --output-format csv -- python -u $GRAFT_REPO_ROOT/tools/bench_observe.py > /dev/null 2>&1 || exit $?
cut -c1-200 $GRAFT_REPO_ROOT/$O/prof/run_kernel_stats.csv
