#!/bin/bash
# Fourier-path bench lines (cfg3, cfg5) and rocprofv3 kernel stats of cfg3.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/fft; mkdir -p $O
timeout -k 10 300 python -u bench.py --config cfg3 --steps 10 --warmup 2 --cpu-seconds ${CPU_S:-10} > $O/cfg3.json 2> $O/cfg3.err || exit $?
cat $O/cfg3.json
timeout -k 10 300 python -u bench.py --config cfg5 --steps 10 --warmup 2 --cpu-seconds ${CPU_S:-10} > $O/cfg5.json 2> $O/cfg5.err || exit $?
cat $O/cfg5.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof3 -o run --output-format csv -- python -u $GRAFT_REPO_ROOT/bench.py --config cfg3 --steps 5 --warmup 1 --cpu-seconds 0 --no-parity > /dev/null 2>&1 || exit $?
head -8 $GRAFT_REPO_ROOT/$O/prof3/run_kernel_stats.csv | cut -c1-220
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof5 -o run --output-format csv -- python -u $GRAFT_REPO_ROOT/bench.py --config cfg5 --steps 5 --warmup 1 --cpu-seconds 0 --no-parity > /dev/null 2>&1 || exit $?
head -8 $GRAFT_REPO_ROOT/$O/prof5/run_kernel_stats.csv | cut -c1-220
