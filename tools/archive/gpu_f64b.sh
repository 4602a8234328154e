#!/bin/bash
# FP64 kernel at MP/NP = 128: its tests, the metric line (regression check) and the cfg4 line.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/f64b; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_f64.py tests/test_gpu_parity.py -x -v --timeout 180 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed|Error|assert" $O/pytest.log | tail -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --cpu-seconds 0 --no-extras > $O/bench.json 2> $O/bench.err || exit $?
cat $O/bench.json
timeout -k 10 300 python -u bench.py --config cfg4 --steps 3 --warmup 1 --cpu-seconds 0 > $O/bench_cfg4.json 2> $O/bench_cfg4.err || exit $?
cat $O/bench_cfg4.json
