#!/bin/bash
# Round-2 evidence: metric bench + rocprof stats, cfg4 bench, cfg3 / cfg5 bench + stats + PMC (k_fft_*).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ev; mkdir -p $O
cd $R
timeout -k 10 400 python -u bench.py > $O/metric.json 2> $O/metric.err || exit $?
cat $O/metric.json
timeout -k 10 300 python -u bench.py --config cfg4 --steps 5 --warmup 1 --cpu-seconds 0 --no-extras > $O/cfg4.json 2> $O/cfg4.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/metric_prof -o run --output-format csv -- python3 $R/bench.py --cpu-seconds 0 --no-extras > $O/metric_prof.json 2> $O/metric_prof.err || exit $?
cd $R
CFG=cfg3 bash tools/pmc_fft.sh || exit $?
CFG=cfg5 bash tools/pmc_fft.sh || exit $?
