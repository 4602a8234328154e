#!/bin/bash
# k_fft_wreg softmax trim: Fourier tests, cfg3 bench (x2) and cfg5
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03l; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -k "fourier or cfg5 or fft or cfg3 or fullbatch" > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; grep -E "FAILED|Error" $O/pytest.log | head -10
[ $rc -ne 0 ] && exit $rc
for c in cfg3 cfg3 cfg5; do
  timeout -k 10 200 python -u bench.py --config $c --steps 10 --warmup 2 --cpu-seconds 0 > $O/$c.json 2> $O/$c.err || exit $?
  python -c "import json;d=json.load(open('$O/$c.json'));print('$c',d['value'],d['roofline']['kernel_ms'],d['roofline']['frac'],d['parity']['rel_fro'])"
done
# per-rank work of the 8-GPU K-shard step: 16 components over the whole batch (prepare share = step - kernel)
timeout -k 10 200 python -u bench.py --components 16 --steps 20 --warmup 3 --cpu-seconds 0 --no-extras --no-parity > $O/k16.json 2> $O/k16.err || exit $?
python -c "import json;d=json.load(open('$O/k16.json'));r=d['roofline'];print('K=16',d['value'],d['ms_per_step'],r['kernel_ms'],round(d['ms_per_step']-r['kernel_ms'],4))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/k16prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --components 16 --steps 10 --warmup 2 --cpu-seconds 0 --no-extras --no-parity > $GRAFT_REPO_ROOT/$O/k16prof.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT && python3 tools/trace_summary.py $(find $O/k16prof -name '*kernel_trace.csv' | head -1) "" | head -14
