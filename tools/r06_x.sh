#!/bin/bash
# Round 6: the K-shard prepare's Cholesky-status copy posted after the table set's event (off the path to the partial
# kernel): emulated world-8 rank step at K = 16 (ranks 0 / 7), world 4 / 2, cfg4; then the K-shard GPU tests.
set -o pipefail
R=$PWD
O=$R/gpurun_out/r06x
mkdir -p $O
for rep in 1 2 3; do
  timeout -k 10 200 python tools/kshard_native_step.py --K 16 --steps 40 --emulate-world 8:0 $( [ $rep = 1 ] || echo --no-parity ) > $O/rank16_r0_$rep.json 2> $O/rank16_r0_$rep.err || exit 1
done
timeout -k 10 200 python tools/kshard_native_step.py --K 16 --steps 40 --emulate-world 8:7 > $O/rank16_r7.json 2> $O/rank16_r7.err || exit 1
timeout -k 10 200 python tools/kshard_native_step.py --K 32 --steps 30 --emulate-world 4:0 > $O/rank32_w4.json 2> $O/rank32_w4.err || exit 1
timeout -k 10 200 python tools/kshard_native_step.py --K 64 --steps 20 --emulate-world 2:0 > $O/rank64_w2.json 2> $O/rank64_w2.err || exit 1
timeout -k 10 200 python tools/kshard_native_step.py --K 32 --N 128 --B 50000 --steps 20 --emulate-world 8:0 > $O/cfg4_rank32.json 2> $O/cfg4_rank32.err || exit 1
timeout -k 10 700 python -u -m pytest tests/test_gpu_kshard_rank.py tests/test_gpu_kshard_native.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
echo done
