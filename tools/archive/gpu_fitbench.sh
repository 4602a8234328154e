#!/bin/bash
# Device EM iteration timing + rocprofv3 kernel stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/fitb; mkdir -p $O
timeout -k 10 300 python -u tools/bench_fit.py > $O/bench.json 2> $O/bench.err || exit $?
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
FIT_CPU_SECONDS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run --output-format csv -- python -u $GRAFT_REPO_ROOT/tools/bench_fit.py > /dev/null 2>&1 || exit $?
cut -c1-160 $GRAFT_REPO_ROOT/$O/prof/run_kernel_stats.csv | head -14
