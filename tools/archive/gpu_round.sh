#!/bin/bash
# One GPU call: parity tests, bench line, rocprofv3 kernel stats of the same bench command.
# usage (on the box, from the repo root): bash tools/gpu_round.sh TAG
set -o pipefail
TAG=${1:-run}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python -u $R/bench.py --cpu-seconds 0 > $O/prof_bench.json 2> $O/prof.err || exit $?
cat $O/prof_bench.json
find $O/prof -name '*kernel_stats.csv' -exec head -6 {} \;
