#!/bin/bash
# Round 4: the library's K-shard step (qce_kshard_*) on the GPU -- world-1 RCCL and 2/3-rank host-transport tests,
# then a kernel trace of the world-1 RCCL metric step (RCCL kernels beside the estimate kernels).
set -o pipefail
mkdir -p gpurun_out/r04a
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_kshard_native.py tests/test_gpu_configs.py -x -v --timeout 170 --timeout-method thread > gpurun_out/r04a/pytest.log 2>&1 || { tail -40 gpurun_out/r04a/pytest.log; exit 1; }
tail -3 gpurun_out/r04a/pytest.log
timeout -k 10 300 python -u tools/kshard_native_step.py > gpurun_out/r04a/step.json 2> gpurun_out/r04a/step.err || { tail -30 gpurun_out/r04a/step.err; exit 1; }
cat gpurun_out/r04a/step.json
# one rank's share of the 8-GPU metric step (K/N = 16 components over the whole batch), 1 and 2 chunks, with and
# without the spare table set (the next prepare overlapping the current step)
for C in 1 2; do for SB in "" "--single-buffer"; do
  timeout -k 10 200 python -u tools/kshard_native_step.py --K 16 --chunks $C --steps 20 $SB >> gpurun_out/r04a/rank16.jsonl 2>> gpurun_out/r04a/rank16.err || { tail -20 gpurun_out/r04a/rank16.err; exit 1; }
done; done
cat gpurun_out/r04a/rank16.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/r04a/prof -o trace -- python3 tools/kshard_native_step.py --steps 5 > gpurun_out/r04a/prof.log 2> gpurun_out/r04a/prof.err || { tail -30 gpurun_out/r04a/prof.err; exit 1; }
find gpurun_out/r04a/prof -name "*kernel_stats.csv" | head -3
timeout -k 10 60 ./tools/probe/mfma_f64_probe > gpurun_out/r04a/mfma_f64_probe.txt 2>&1 || true
cat gpurun_out/r04a/mfma_f64_probe.txt
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 rocprofv3 -L > gpurun_out/r04a/counters_list.txt 2>&1 || true
grep -i -E "DRAM|MALL|EA0_RD|EA_RD|HBM" gpurun_out/r04a/counters_list.txt | head -40
#!/bin/bash
# Round 4: A/B of the FP64 headline kernel's launch shape (8-wave workgroup vs two 4-wave workgroups per CU), each
# with its parity line, then the FP64 tests under the new shape.
set -o pipefail
mkdir -p gpurun_out/r04b
for V in 8:0 42:0 8:1 42:1 8:0 42:0 8:1 42:1; do
  W=${V%:*}; P=${V#*:}
  QCE_F64_WAVES=$W QCE_F64_PIPE=$P timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --cpu-seconds 0 --no-extras > gpurun_out/r04b/bench_w${W}p$P.json 2> gpurun_out/r04b/bench_w${W}p$P.err || { tail -20 gpurun_out/r04b/bench_w${W}p$P.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r04b/bench_w${W}p$P.json'));r=d['roofline'];print('W=$W P=$P', d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], r.get('mfma_issue_frac'), d['parity']['rel_fro'])"
done
QCE_F64_WAVES=42 QCE_F64_PIPE=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_f64.py tests/test_gpu_fullbatch.py tests/test_gpu_argmax_metric.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04b/pytest42.log 2>&1 || { tail -30 gpurun_out/r04b/pytest42.log; exit 1; }
tail -2 gpurun_out/r04b/pytest42.log
