#!/bin/bash
# rocprofv3 --kernel-trace --stats of the other configurations' bench commands (this build), one run each under its
# own time limit: the kernel averages beside the HIP-event kernel_ms of each line.
set -o pipefail
R=$PWD
mkdir -p gpurun_out/r05s2
cd /tmp && export TMPDIR=/tmp
for spec in "cfg2:" "cfg3:" "cfg5:" "cfg3:--mean" "cfg5:--mean" "cfg4:"; do
  c=${spec%%:*}; x=${spec#*:}; tag=$c${x:+_mean}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r05s2/$tag -o run --output-format csv -- python3 $R/bench.py --config $c $x --no-extras --cpu-seconds 0 > $R/gpurun_out/r05s2/$tag.json 2> $R/gpurun_out/r05s2/$tag.err || exit $?
done
