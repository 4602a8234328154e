#!/bin/bash
# One GPU call: A/B of the estimate-kernel variants, then the PMC passes of the bench command.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
timeout -k 10 200 python -u tools/ab_variants.py > gpurun_out/ab.log 2>&1 || exit $?
cat gpurun_out/ab.log
timeout -k 10 900 bash tools/profile_pmc.sh || exit $?
python tools/pmc_summary.py gpurun_out/pmc k_est_all_h2 metric 100000 h2 gpurun_out/traffic_metric.json
