#!/bin/bash
# Host-side submission time of the K-shard rank step (is the host running ahead of the GPU?), emulated world 8.
set -o pipefail
O=$PWD/gpurun_out/r06o
mkdir -p $O
timeout -k 10 200 python tools/kshard_native_step.py --K 16 --steps 40 --emulate-world 8:0 --no-parity > $O/rank16_host.json 2>&1 || exit 1
QCE_KSHARD_USED_ON_CS=1 timeout -k 10 200 python tools/kshard_native_step.py --K 16 --steps 40 --emulate-world 8:0 --no-parity > $O/rank16_host_oc1.json 2>&1 || exit 1
echo done
