#!/bin/bash
# Round 6: the K-shard prepare's tail (filter, packs, status copy, shift) on the compute stream behind the
# factorisation (default) vs the whole prepare on the prepare stream (QCE_KSHARD_PREP_TAIL=0): emulated world-8 rank
# step at K = 16, interleaved; then the K-shard / config / parity GPU tests on the default.
set -o pipefail
R=$PWD
O=$R/gpurun_out/r06z
mkdir -p $O
for rep in 1 2 3; do
  for pt in 1 0; do
    QCE_KSHARD_PREP_TAIL=$pt timeout -k 10 200 python tools/kshard_native_step.py --K 16 --steps 40 --emulate-world 8:0 $( [ $rep = 1 ] || echo --no-parity ) > $O/rank16_pt${pt}_$rep.json 2> $O/rank16_pt${pt}_$rep.err || exit 1
  done
done
timeout -k 10 200 python tools/kshard_native_step.py --K 16 --steps 40 --emulate-world 8:7 > $O/rank16r7_pt1.json 2> $O/rank16r7_pt1.err || exit 1
timeout -k 10 200 python tools/kshard_native_step.py --K 32 --N 128 --B 50000 --steps 20 --emulate-world 8:0 > $O/cfg4_pt1.json 2> $O/cfg4_pt1.err || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_kshard_rank.py tests/test_gpu_kshard_native.py tests/test_gpu_configs.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
echo done
