#!/bin/bash
# Round 6: the K-shard row passes beside the next prepare (send-row scaling, finalisation) with a capped grid
# (QCE_KSHARD_ROWPASS_WG; 16-byte accesses in the scaling): emulated world-8 rank step at K = 16, interleaved A/B,
# then the rank parity tests on the default.
set -o pipefail
R=$PWD
O=$R/gpurun_out/r06u
mkdir -p $O
for rep in 1 2; do
  for wg in 0 256 512 1024 2048; do
    QCE_KSHARD_ROWPASS_WG=$wg timeout -k 10 200 python tools/kshard_native_step.py --K 16 --steps 40 --emulate-world 8:0 --no-parity > $O/rank16_wg${wg}_$rep.json 2> $O/rank16_wg${wg}_$rep.err || exit 1
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_kshard_rank.py tests/test_gpu_kshard_native.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
tail -2 $O/pytest.log
echo done
