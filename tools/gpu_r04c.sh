#!/bin/bash
# Round 4: the library's K-shard tests after the prepare-overlap fix, one rank's share of the 8-GPU metric step
# (K/N = 16) with / without the spare table set, cfg4 (K=256, N=128) bench line and its per-rank K-shard steps
# (K_local = 128/64/32 over all 5e4 rows, 1 and 2 chunks), then PMC passes of k_est_all_f64 at cfg4.
set -o pipefail
mkdir -p gpurun_out/r04c
timeout -k 10 400 python -u -m pytest tests/test_gpu_kshard_native.py -x -q --timeout 170 --timeout-method thread > gpurun_out/r04c/pytest.log 2>&1 || { tail -40 gpurun_out/r04c/pytest.log; exit 1; }
tail -2 gpurun_out/r04c/pytest.log
for C in 1 2; do for SB in "" "--single-buffer"; do
  timeout -k 10 200 python -u tools/kshard_native_step.py --K 16 --chunks $C --steps 30 $SB 2>> gpurun_out/r04c/rank16.err | tail -1 >> gpurun_out/r04c/rank16.jsonl || { tail -20 gpurun_out/r04c/rank16.err; exit 1; }
done; done
cat gpurun_out/r04c/rank16.jsonl
timeout -k 10 300 python -u bench.py --config cfg4 --steps 10 --warmup 2 --cpu-seconds 0 > gpurun_out/r04c/cfg4.json 2> gpurun_out/r04c/cfg4.err || { tail -20 gpurun_out/r04c/cfg4.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r04c/cfg4.json'));r=d['roofline'];print('cfg4', d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], r.get('mfma_issue_frac'), d['parity']['rel_fro'])"
for K in 128 64 32; do for C in 1 2; do
  timeout -k 10 200 python -u tools/kshard_native_step.py --K $K --N 128 --B 50000 --chunks $C --steps 10 2>> gpurun_out/r04c/rank_cfg4.err | tail -1 >> gpurun_out/r04c/rank_cfg4.jsonl || { tail -20 gpurun_out/r04c/rank_cfg4.err; exit 1; }
done; done
cat gpurun_out/r04c/rank_cfg4.jsonl
CFG=cfg4 KPAT=k_est_all_f64 CAL=1 TAG=cfg4 bash tools/pmc_kernel.sh
