#!/bin/bash
# A/B: the double-buffered K-shard's next prepare waiting for the step's kernels on the compute stream (new) vs the
# step's close on the communication stream (QCE_KSHARD_USED_ON_CS=1, round 5), emulated world-8 rank 0 at K=16;
# single buffer beside; then a kernel trace of the new order.
set -o pipefail
R=$PWD
O=$R/gpurun_out/r06n
mkdir -p $O
for rep in 1 2; do
  for oc in 0 1; do
    QCE_KSHARD_USED_ON_CS=$oc timeout -k 10 200 python tools/kshard_native_step.py --K 16 --steps 40 --emulate-world 8:0 --no-parity > $O/rank16_oc${oc}_$rep.json 2>&1 || exit 1
  done
  timeout -k 10 200 python tools/kshard_native_step.py --K 16 --steps 40 --emulate-world 8:0 --no-parity --single-buffer > $O/rank16_single_$rep.json 2>&1 || exit 1
done
timeout -k 10 200 python tools/kshard_native_step.py --K 16 --steps 20 --emulate-world 8:0 > $O/rank16_parity.json 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr16 -o run --output-format csv -- python3 $R/tools/kshard_native_step.py --K 16 --steps 30 --emulate-world 8:0 --no-parity > $O/tr16.json 2> $O/tr16.err || exit 1
echo done
