#!/bin/bash
# Prepare-path check: prepare-sensitive GPU tests, then kernel stats of the metric and cfg4 commands.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/prep; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_quirks.py tests/test_gpu_f64.py -m gpu -x -q --timeout 180 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $O/pytest.log | tail -8; [ $rc -ne 0 ] && exit $rc
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 -u bench.py --steps 10 --warmup 2 --cpu-seconds 0 --no-extras > $O/bench.json 2> $O/prof.log || exit $?
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/kernel_stats.csv
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof4 -o run --output-format csv -- python3 -u bench.py --config cfg4 --steps 3 --warmup 1 --cpu-seconds 0 > $O/bench4.json 2> $O/prof4.log || exit $?
find $O/prof4 -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/kernel_stats4.csv
python3 - <<'PY'
import csv, json
for b in ('gpurun_out/prep/bench.json', 'gpurun_out/prep/bench4.json'):
    L = [l for l in open(b) if l.startswith('{')]; d = json.loads(L[-1]); r = d['roofline']
    print(b, d['value'], d['ms_per_step'], r['kernel_ms'], d['parity']['rel_fro'])
for f in ('gpurun_out/prep/kernel_stats.csv','gpurun_out/prep/kernel_stats4.csv'):
    print(f)
    for x in list(csv.DictReader(open(f)))[:14]:
        print(f"  {x['Name'].split('(')[0][:48]:48s} {x['Calls']:>4} {float(x['AverageNs'])/1e3:9.1f} us {float(x['Percentage']):6.2f}%")
PY
