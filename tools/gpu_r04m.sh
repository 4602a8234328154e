#!/bin/bash
# Round 4: k_est_all_f64 with row-split wave pairs at padded 128 x 128 (cfg4): parity tests of the N = 128 paths
# first, then cfg4 / metric bench lines, then the whole GPU suite.  Outputs under gpurun_out/r04m/.
set -o pipefail
O=gpurun_out/r04m
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > $O/configs.log 2>&1 || { tail -40 $O/configs.log; exit 1; }
tail -2 $O/configs.log
for C in cfg4 metric cfg4; do
  timeout -k 10 300 python -u bench.py --config $C --steps 10 --warmup 2 --cpu-seconds 0 --no-extras > $O/$C.json 2> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$C.json'));r=d['roofline'];print('$C', d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], r.get('mfma_issue_frac'), d['parity']['rel_fro'])" | tee -a $O/ab.txt
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
