#!/bin/bash
# Round 4: the K-shard step with the control communicator and alternating send buffers (step t's collectives beside
# step t+1's kernels): library K-shard tests, per-rank step timings (K/N = 16 metric share; cfg4 shares), an RCCL
# debug log of the world-1 collectives, then the deeper-ring checks (cfg4 / metric lines, FP64 tests).
set -o pipefail
mkdir -p gpurun_out/r04e
timeout -k 10 400 python -u -m pytest tests/test_gpu_kshard_native.py -x -q --timeout 170 --timeout-method thread > gpurun_out/r04e/pytest.log 2>&1 || { tail -40 gpurun_out/r04e/pytest.log; exit 1; }
tail -2 gpurun_out/r04e/pytest.log
for C in 1 2; do for SB in "" "--single-buffer"; do
  timeout -k 10 200 python -u tools/kshard_native_step.py --K 16 --chunks $C --steps 30 $SB 2>> gpurun_out/r04e/rank16.err | tail -1 >> gpurun_out/r04e/rank16.jsonl || { tail -20 gpurun_out/r04e/rank16.err; exit 1; }
done; done
cat gpurun_out/r04e/rank16.jsonl
for K in 32 64 128; do
  timeout -k 10 200 python -u tools/kshard_native_step.py --K $K --N 128 --B 50000 --chunks 2 --steps 10 2>> gpurun_out/r04e/rank_cfg4.err | tail -1 >> gpurun_out/r04e/rank_cfg4.jsonl || { tail -20 gpurun_out/r04e/rank_cfg4.err; exit 1; }
done
cat gpurun_out/r04e/rank_cfg4.jsonl
NCCL_DEBUG=INFO NCCL_DEBUG_SUBSYS=INIT,COLL timeout -k 10 200 python -u tools/kshard_native_step.py --K 16 --B 20000 --steps 2 > gpurun_out/r04e/rccl_debug.log 2>&1 || { tail -20 gpurun_out/r04e/rccl_debug.log; exit 1; }
grep -c -E "AllReduce|ReduceScatter|AllGather" gpurun_out/r04e/rccl_debug.log || true
bash tools/gpu_r04d.sh
