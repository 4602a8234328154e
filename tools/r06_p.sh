#!/bin/bash
# A/B of the K-shard prepare scheduling at emulated world 8 (K=16): per-set prepare streams + set release on the
# compute stream (new), one prepare stream (QCE_KSHARD_ONE_PS=1), and the round-5 order (both env switches);
# a kernel trace of the new order; the K-shard GPU tests.
set -o pipefail
R=$PWD
O=$R/gpurun_out/r06p
mkdir -p $O
for rep in 1 2; do
  timeout -k 10 200 python tools/kshard_native_step.py --K 16 --steps 40 --emulate-world 8:0 --no-parity > $O/rank16_new_$rep.json 2>&1 || exit 1
  QCE_KSHARD_ONE_PS=1 timeout -k 10 200 python tools/kshard_native_step.py --K 16 --steps 40 --emulate-world 8:0 --no-parity > $O/rank16_oneps_$rep.json 2>&1 || exit 1
  QCE_KSHARD_ONE_PS=1 QCE_KSHARD_USED_ON_CS=1 timeout -k 10 200 python tools/kshard_native_step.py --K 16 --steps 40 --emulate-world 8:0 --no-parity > $O/rank16_r05_$rep.json 2>&1 || exit 1
done
timeout -k 10 300 python tools/kshard_native_step.py --K 32 --N 128 --B 50000 --steps 10 --emulate-world 8:0 --no-parity > $O/rank_cfg4_new.json 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_kshard_rank.py tests/test_gpu_kshard_native.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr16 -o run --output-format csv -- python3 $R/tools/kshard_native_step.py --K 16 --steps 30 --emulate-world 8:0 --no-parity > $O/tr16.json 2> $O/tr16.err || exit 1
echo done
