#!/bin/bash
# Round 4: cfg4 (K=256, N=128): bench line, PMC passes of k_est_all_f64 at N=128 (traffic JSON for this build), and
# the per-rank K-shard step of a 2/4/8-GPU split (K_local = 128/64/32 over all 5e4 rows), 1 and 2 chunks.
set -o pipefail
mkdir -p gpurun_out/r04c
for P in 0 1 0 1; do
  QCE_F64_PIPE=$P timeout -k 10 300 python -u bench.py --config cfg4 --steps 10 --warmup 2 --cpu-seconds 0 > gpurun_out/r04c/cfg4_p$P.json 2> gpurun_out/r04c/cfg4.err || { tail -20 gpurun_out/r04c/cfg4.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r04c/cfg4_p$P.json'));r=d['roofline'];print('cfg4 P=$P', d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], r.get('mfma_issue_frac'), d['parity']['rel_fro'])"
done
QCE_F64_PIPE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_f64.py tests/test_gpu_configs.py -x -q --timeout 150 --timeout-method thread > gpurun_out/r04c/pytest_pipe.log 2>&1 || { tail -30 gpurun_out/r04c/pytest_pipe.log; exit 1; }
tail -2 gpurun_out/r04c/pytest_pipe.log
for K in 128 64 32; do for C in 1 2; do
  timeout -k 10 200 python -u tools/kshard_native_step.py --K $K --N 128 --B 50000 --chunks $C --steps 10 >> gpurun_out/r04c/rank_cfg4.jsonl 2>> gpurun_out/r04c/rank_cfg4.err || { tail -20 gpurun_out/r04c/rank_cfg4.err; exit 1; }
done; done
cat gpurun_out/r04c/rank_cfg4.jsonl
CFG=cfg4 KPAT=k_est_all_f64 CAL=1 TAG=cfg4 bash tools/pmc_kernel.sh
