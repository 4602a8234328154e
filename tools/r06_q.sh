#!/bin/bash
# K-shard rank step (emulated world 8, K=16) with more HIP hardware queues per process (streams beyond
# GPU_MAX_HW_QUEUES share a hardware queue and serialise): new prepare order vs round-5 order, 4 / 8 / 16 queues.
set -o pipefail
R=$PWD
O=$R/gpurun_out/r06q
mkdir -p $O
for rep in 1 2; do
  for q in 4 8 16; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python tools/kshard_native_step.py --K 16 --steps 40 --emulate-world 8:0 --no-parity > $O/rank16_new_q${q}_$rep.json 2>&1 || exit 1
    GPU_MAX_HW_QUEUES=$q QCE_KSHARD_ONE_PS=1 QCE_KSHARD_USED_ON_CS=1 timeout -k 10 200 python tools/kshard_native_step.py --K 16 --steps 40 --emulate-world 8:0 --no-parity > $O/rank16_r05_q${q}_$rep.json 2>&1 || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr16 -o run --output-format csv -- python3 $R/tools/kshard_native_step.py --K 16 --steps 30 --emulate-world 8:0 --no-parity > $O/tr16.json 2> $O/tr16.err || exit 1
echo done
