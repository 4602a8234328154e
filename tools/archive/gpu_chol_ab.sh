#!/bin/bash
# M <= 64 Cholesky kernel A/B (QCE_CHOL = wave | lds | tri): table parity tests, then rocprof of the metric bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/cholab; mkdir -p $O
cd $R
for v in wave lds tri; do
  QCE_CHOL=$v timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "table or prepare or golden or quirk or f64" > $O/pytest_$v.log 2>&1
  rc=$?; echo "$v: $(tail -1 $O/pytest_$v.log)"; [ $rc -ne 0 ] && exit $rc
done
cd /tmp && export TMPDIR=/tmp
for v in wave lds tri; do
  QCE_CHOL=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run --output-format csv -- python3 $R/bench.py --cpu-seconds 0 --no-extras --no-parity --steps 10 > $O/bench_$v.json 2> $O/bench_$v.err || exit $?
  python3 -c "
import csv, json
d = json.load(open('$O/bench_$v.json')); print('$v value', d['value'], 'ms_per_step', d['ms_per_step'])
for r in csv.DictReader(open('$O/prof_$v/run_kernel_stats.csv')):
    if 'chol' in r['Name']: print('   ', r['Name'][:40], round(float(r['AverageNs'])/1e3, 1), 'us')
"
done
