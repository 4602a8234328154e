#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/scm; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_scm.py tests/test_baselines.py -m gpu -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; grep -E "PASSED|FAILED|passed|failed|Error" $O/pytest.log | tail -20; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/bench_scm.py > $O/bench.json 2> $O/bench.err || exit $?
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
SCM_B=20000 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run --output-format csv -- python -u $GRAFT_REPO_ROOT/tools/bench_scm.py > /dev/null 2>&1 || exit $?
cut -c1-150 $GRAFT_REPO_ROOT/$O/prof/run_kernel_stats.csv | head -5
