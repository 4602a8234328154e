#!/bin/bash
# Round 6: the two-phase blocked pair Cholesky (k_chol_inv_lds3) vs the one-phase pair kernel (QCE_CHOL_V3=0):
# tables and prepare times, the prepare-table parity tests, the emulated world-8 rank step.
set -o pipefail
R=$PWD
O=$R/gpurun_out/r06r
mkdir -p $O
timeout -k 10 600 python tools/chol_pairs_check.py --env QCE_CHOL_V3 > $O/chol_v3.jsonl 2> $O/chol_v3.err || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_golden_bench_configs.py tests/test_gpu_kshard_native.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
for rep in 1 2; do
  timeout -k 10 200 python tools/kshard_native_step.py --K 16 --steps 40 --emulate-world 8:0 --no-parity > $O/rank16_v3_$rep.json 2>&1 || exit 1
  QCE_CHOL_V3=0 timeout -k 10 200 python tools/kshard_native_step.py --K 16 --steps 40 --emulate-world 8:0 --no-parity > $O/rank16_v2_$rep.json 2>&1 || exit 1
done
echo done
