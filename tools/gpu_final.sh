#!/bin/bash
# Round-end evidence for the current tree: the driver's bench command, its rocprofv3 kernel trace + stats (csv, the
# same command), the PMC passes of the headline kernel with K=1 calibration and DRAM requests (traffic JSON stamped
# with this build's id), a bench line with that traffic, the GPU suite and smoke(). Outputs under gpurun_out/final/.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/final
cd $R
timeout -k 10 400 python -u bench.py > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err || { tail -20 gpurun_out/final/bench.err; exit 1; }
cat gpurun_out/final/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/final/prof -o run --output-format csv -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $R/gpurun_out/final/prof.log 2> $R/gpurun_out/final/prof.err || { tail -20 $R/gpurun_out/final/prof.err; exit 1; }
cd $R
grep -c -i -E "signal|abort" gpurun_out/final/prof.err || true
find gpurun_out/final/prof -name "*kernel_stats.csv" -exec head -4 {} \; | cut -c1-200
CFG=metric KPAT=k_est_all_f64 CAL=1 TAG=metric bash tools/pmc_kernel.sh || exit 1
cp gpurun_out/pmc_metric/traffic_metric.json profiles/traffic_metric.json
timeout -k 10 400 python -u bench.py --cpu-seconds 0 --no-extras > gpurun_out/final/bench_traffic.json 2> gpurun_out/final/bench_traffic.err || { tail -20 gpurun_out/final/bench_traffic.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/final/bench_traffic.json'));print(json.dumps(d['roofline']))"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/final/pytest.log 2>&1 || { tail -30 gpurun_out/final/pytest.log; exit 1; }
tail -2 gpurun_out/final/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || { tail -20 gpurun_out/final/smoke.log; exit 1; }
tail -3 gpurun_out/final/smoke.log
