#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab2
for rep in 1 2; do
for lib in libqce_old.so libqce.so; do
  QCE_LIB=quantized_channel_estimation_amd/$lib timeout -k 10 200 python -u bench.py --config cfg3 --steps 30 --warmup 3 --cpu-seconds 0 --no-extras --no-parity > gpurun_out/ab2/$lib.$rep.json 2>/dev/null || exit $?
  python -c "import json;d=json.load(open('gpurun_out/ab2/$lib.$rep.json'));print('$lib', $rep, d['roofline']['kernel_ms'])"
done
done
