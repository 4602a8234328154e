#!/bin/bash
# Full GPU pass: whole GPU suite, smoke, metric + cfg4 lines, 2-rank K-shard rehearsal (gloo on one GPU),
# rocprof kernel stats of the metric command.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/full; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $O/pytest.log | tail -8; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));r=d['roofline'];print('metric',d['value'],d['ms_per_step'],r['kernel_ms'],r['frac'],r['mfma_issue_frac'],d['parity']['rel_fro'], d['cpu_baseline']['value'], d['fast_path']['value'], d['dropin']['value'])"
timeout -k 10 300 python -u bench.py --config cfg4 --steps 3 --warmup 1 --cpu-seconds 0 > $O/bench4.json 2> $O/bench4.err || exit $?
python3 -c "import json;d=json.load(open('$O/bench4.json'));r=d['roofline'];print('cfg4',d['value'],d['ms_per_step'],r['kernel_ms'],r['frac'],r['mfma_issue_frac'],d['parity']['rel_fro'])"
timeout -k 10 300 python -u bench.py --gpus 2 --backend gloo --collective ar --steps 3 --warmup 1 --batch 20000 > $O/bench_k2.json 2> $O/bench_k2.err || { tail -20 $O/bench_k2.err; exit 1; }
python3 -c "import json;L=[l for l in open('$O/bench_k2.json') if l.startswith('{')];d=json.loads(L[-1]);print('k2 gloo',d['value'],d['parity']['rel_fro'])"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 -u bench.py --steps 10 --warmup 2 --cpu-seconds 0 --no-parity --no-extras > $O/prof.log 2>&1 || exit $?
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/kernel_stats.csv
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof4 -o run --output-format csv -- python3 -u bench.py --config cfg4 --steps 3 --warmup 1 --cpu-seconds 0 --no-parity > $O/prof4.log 2>&1 || exit $?
find $O/prof4 -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/kernel_stats4.csv
python3 - <<'PY'
import csv
for f in ('gpurun_out/full/kernel_stats.csv','gpurun_out/full/kernel_stats4.csv'):
    print(f)
    for x in list(csv.DictReader(open(f)))[:12]:
        print(f"  {x['Name'].split('(')[0][:48]:48s} {x['Calls']:>4} {float(x['AverageNs'])/1e3:9.1f} us {float(x['Percentage']):6.2f}%")
PY
