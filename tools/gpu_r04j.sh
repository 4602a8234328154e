#!/bin/bash
# Round 4, after the inline-asm LDS DMA: segment stamps (metric, cfg4), prefetch distance A/B (E = 4 / 6 / 8,
# libqce_e4/e8.so via QCE_LIB), per-rank K-shard steps (metric K = 16; cfg4 K = 32 / 64 / 128), block-loop probe.
set -o pipefail
O=gpurun_out/r04j
mkdir -p $O
L=quantized_channel_estimation_amd
for C in metric cfg4; do
  QCE_LIB=$L/libqce_stamps.so timeout -k 10 300 python -u tools/f64_stamps.py $C > $O/stamps_$C.txt 2>&1 || { tail -20 $O/stamps_$C.txt; exit 1; }
  grep -v amdgpu.ids $O/stamps_$C.txt
done
for r in 1 2; do for V in libqce libqce_e4 libqce_e8; do for C in metric cfg4; do
  QCE_LIB=$L/$V.so timeout -k 10 300 python -u bench.py --config $C --steps 8 --warmup 2 --cpu-seconds 0 --no-extras > $O/${V}_$C.json 2> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
  python3 -c "import json;d=json.load(open('$O/${V}_$C.json'));r=d['roofline'];print('$V $C', d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], r.get('mfma_issue_frac'), d['parity']['rel_fro'])" | tee -a $O/ab.txt
done; done; done
for C in 1 2; do for SB in "" "--single-buffer"; do
  timeout -k 10 200 python -u tools/kshard_native_step.py --K 16 --chunks $C --steps 30 $SB 2>> $O/rank16.err | tail -1 >> $O/rank16.jsonl || { tail -20 $O/rank16.err; exit 1; }
done; done
cat $O/rank16.jsonl
for K in 128 64 32; do for C in 1 2; do
  timeout -k 10 200 python -u tools/kshard_native_step.py --K $K --N 128 --B 50000 --chunks $C --steps 10 2>> $O/rank_cfg4.err | tail -1 >> $O/rank_cfg4.jsonl || { tail -20 $O/rank_cfg4.err; exit 1; }
done; done
cat $O/rank_cfg4.jsonl
timeout -k 10 60 tools/probe/f64_block_probe > $O/block_probe.txt 2>&1 && cat $O/block_probe.txt
