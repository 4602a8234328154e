#!/bin/bash
# Round 6: Cy / gains / Cr formed inside the factorisation kernel and its status stored straight to pinned memory
# (QCE_CHOL_FUSE_GAIN=0: the separate k_gain_cr launch, A/B): tables, prepare times, the parity tests, bench lines
# of the small configs and the emulated rank step.
set -o pipefail
R=$PWD
O=$R/gpurun_out/r06s
mkdir -p $O
timeout -k 10 600 python tools/chol_pairs_check.py --env QCE_CHOL_FUSE_GAIN > $O/fuse.jsonl 2> $O/fuse.err || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_golden_bench_configs.py tests/test_gpu_kshard_native.py tests/test_gpu_kshard_rank.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
for c in cfg1 cfg2 metric; do
  timeout -k 10 300 python bench.py --config $c --no-extras --cpu-seconds 0 > $O/${c}_bench.json 2> $O/${c}_bench.err || exit 1
  QCE_CHOL_FUSE_GAIN=0 timeout -k 10 300 python bench.py --config $c --no-extras --cpu-seconds 0 > $O/${c}_bench_unfused.json 2> $O/${c}_bench_unfused.err || exit 1
done
for rep in 1 2; do
  timeout -k 10 200 python tools/kshard_native_step.py --K 16 --steps 40 --emulate-world 8:0 --no-parity > $O/rank16_fused_$rep.json 2>&1 || exit 1
  QCE_CHOL_FUSE_GAIN=0 timeout -k 10 200 python tools/kshard_native_step.py --K 16 --steps 40 --emulate-world 8:0 --no-parity > $O/rank16_unfused_$rep.json 2>&1 || exit 1
done
echo done
