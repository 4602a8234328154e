#!/bin/bash
# A/B of the LDS-DMA issue form in k_est_all_f64 (inline-asm global_load_lds: no compiler vmcnt(0) before the next
# LDS read): metric and cfg4 bench lines, then the GPU suite.  Outputs under gpurun_out/r04i/.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04i
mkdir -p $O
cd $R
timeout -k 10 300 python -u bench.py --cpu-seconds 0 > $O/metric.json 2> $O/metric.err || { tail -20 $O/metric.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/metric.json'));r=d['roofline'];print('metric',d['value'],d['ms_per_step'],r['kernel_ms'],r['frac'],r['mfma_issue_frac'],d['parity']['rel_fro'],'fast',d['fast_path']['value'],d['fast_path']['kernel_ms'],d['fast_path']['parity_rel_fro'])"
timeout -k 10 300 python -u bench.py --config cfg4 --cpu-seconds 0 --no-extras > $O/cfg4.json 2> $O/cfg4.err || { tail -20 $O/cfg4.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/cfg4.json'));r=d['roofline'];print('cfg4',d['value'],d['ms_per_step'],r['kernel_ms'],r['frac'],r['mfma_issue_frac'],d['parity']['rel_fro'])"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
