#!/bin/bash
# Round 4, final build: per-rank K-shard steps through qce_kshard_* (world-1 RCCL): metric K = 16 of 128 (8 ranks),
# cfg4 K = 128 / 64 / 32 of 256 (2 / 4 / 8 ranks); chunks 1 and 2, double-buffered (and single-buffered at metric).
set -o pipefail
O=gpurun_out/r04n
mkdir -p $O
for C in 1 2; do for SB in "" "--single-buffer"; do
  timeout -k 10 200 python -u tools/kshard_native_step.py --K 16 --chunks $C --steps 30 $SB 2>> $O/rank16.err | tail -1 >> $O/rank16.jsonl || { tail -20 $O/rank16.err; exit 1; }
done; done
cat $O/rank16.jsonl
for K in 128 64 32; do for C in 1 2; do
  timeout -k 10 200 python -u tools/kshard_native_step.py --K $K --N 128 --B 50000 --chunks $C --steps 10 2>> $O/rank_cfg4.err | tail -1 >> $O/rank_cfg4.jsonl || { tail -20 $O/rank_cfg4.err; exit 1; }
done; done
cat $O/rank_cfg4.jsonl
