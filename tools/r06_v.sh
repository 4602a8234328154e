#!/bin/bash
# Round 6: the K-shard step with M* agreed before the partial kernel (QCE_KSHARD_AGREE_FIRST=1: the compute stream
# waits for the shift MAX, the partial writes rows shifted by M*, no scaling pass) against the default (rows shifted by
# M_r, scaled by e^{M_r - M*} on the comm stream) and the world-1 probe that only skips the scaling (=2): emulated
# world-8 rank step at K = 16, interleaved; then the K-shard GPU tests under AGREE_FIRST=1.
set -o pipefail
R=$PWD
O=$R/gpurun_out/r06v
mkdir -p $O
for rep in 1 2 3; do
  for af in 0 1 2; do
    QCE_KSHARD_AGREE_FIRST=$af timeout -k 10 200 python tools/kshard_native_step.py --K 16 --steps 40 --emulate-world 8:0 $( [ $rep = 1 ] || echo --no-parity ) > $O/rank16_af${af}_$rep.json 2> $O/rank16_af${af}_$rep.err || exit 1
  done
done
QCE_KSHARD_AGREE_FIRST=1 timeout -k 10 200 python tools/kshard_native_step.py --K 32 --N 128 --B 50000 --steps 20 --emulate-world 8:0 > $O/cfg4_af1.json 2> $O/cfg4_af1.err || exit 1
timeout -k 10 200 python tools/kshard_native_step.py --K 32 --N 128 --B 50000 --steps 20 --emulate-world 8:0 > $O/cfg4_af0.json 2> $O/cfg4_af0.err || exit 1
QCE_KSHARD_AGREE_FIRST=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_kshard_rank.py tests/test_gpu_kshard_native.py -x -q --timeout 200 --timeout-method thread > $O/pytest_af1.log 2>&1 || { tail -30 $O/pytest_af1.log; exit 1; }
tail -2 $O/pytest_af1.log
echo done
