#!/bin/bash
# Prepare-kernel timing at the metric config (rocprof stats) + the parity tests that pin the tables.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prepab; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "${SEL:-table or prepare or golden or quirk}" > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --cpu-seconds 0 --no-extras --no-parity --steps 10 > $O/bench.json 2> $O/bench.err || exit $?
python3 -c "
import csv, json
d = json.load(open('$O/bench.json')); print('value', d['value'], 'ms_per_step', d['ms_per_step'])
for r in csv.DictReader(open('$O/prof/run_kernel_stats.csv')):
    if 'chol' in r['Name'] or 'k_est_all_f64' in r['Name']: print(r['Name'][:40], round(float(r['AverageNs'])/1e3, 1), 'us')
"
