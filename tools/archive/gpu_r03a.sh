#!/bin/bash
# Round-3 first box: full GPU suite, smoke, the driver's bench command, rocprof kernel stats of that exact command.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03a; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; grep -E "FAILED|Error" $O/pytest.log | head -5; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit $?
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $O/prof_bench.json 2> $O/prof.err || exit $?
find $O/prof -name "*kernel_stats.csv" | head -3
