#!/bin/bash
# Cholesky/inverse index tables: prepare-table parity tests, metric bench, K=16 per-rank bench with its trace
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03m; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -k "parity or quirk or f64 or configs or kshard" > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; grep -E "FAILED|Error" $O/pytest.log | head -10
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-seconds 0 --no-extras > $O/metric.json 2> $O/metric.err || exit $?
python -c "import json;d=json.load(open('$O/metric.json'));r=d['roofline'];print('metric',d['value'],d['ms_per_step'],r['kernel_ms'],round(d['ms_per_step']-r['kernel_ms'],4),d['parity']['rel_fro'])"
timeout -k 10 200 python -u bench.py --components 16 --steps 20 --warmup 3 --cpu-seconds 0 --no-extras --no-parity > $O/k16.json 2> $O/k16.err || exit $?
python -c "import json;d=json.load(open('$O/k16.json'));r=d['roofline'];print('K=16',d['value'],d['ms_per_step'],r['kernel_ms'],round(d['ms_per_step']-r['kernel_ms'],4))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/k16prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --components 16 --steps 10 --warmup 2 --cpu-seconds 0 --no-extras --no-parity > $GRAFT_REPO_ROOT/$O/k16prof.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT && python3 tools/trace_summary.py $(find $O/k16prof -name '*kernel_trace.csv' | head -1) "" | head -8
