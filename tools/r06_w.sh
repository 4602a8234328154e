#!/bin/bash
# Round 6: RCCL's PreMulSum reduce-scatter where a one-time check on the communicator finds it exact (the scaling
# rides the collective; default) against the scaling kernel + SUM (QCE_KSHARD_RS_PREMUL=0): emulated world-8 rank step
# at K = 16 (ranks 0 and 7) and cfg4 K = 32, interleaved; the single-buffered step as a data point; then the K-shard
# GPU tests on the default.
set -o pipefail
R=$PWD
O=$R/gpurun_out/r06w
mkdir -p $O
for rep in 1 2 3; do
  for pm in 1 0; do
    QCE_KSHARD_RS_PREMUL=$pm timeout -k 10 200 python tools/kshard_native_step.py --K 16 --steps 40 --emulate-world 8:0 $( [ $rep = 1 ] || echo --no-parity ) > $O/rank16_pm${pm}_$rep.json 2> $O/rank16_pm${pm}_$rep.err || exit 1
  done
done
for pm in 1 0; do
  QCE_KSHARD_RS_PREMUL=$pm timeout -k 10 200 python tools/kshard_native_step.py --K 16 --steps 40 --emulate-world 8:7 > $O/rank16r7_pm${pm}.json 2> $O/rank16r7_pm${pm}.err || exit 1
  QCE_KSHARD_RS_PREMUL=$pm timeout -k 10 200 python tools/kshard_native_step.py --K 32 --N 128 --B 50000 --steps 20 --emulate-world 8:0 > $O/cfg4_pm${pm}.json 2> $O/cfg4_pm${pm}.err || exit 1
done
timeout -k 10 200 python tools/kshard_native_step.py --K 16 --steps 40 --emulate-world 8:0 --single-buffer --no-parity > $O/rank16_single.json 2> $O/rank16_single.err || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_kshard_rank.py tests/test_gpu_kshard_native.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
echo done
