#!/bin/bash
# GPU parity tests only (optionally a -k expression), one process, per-test timeout.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
K=${1:-}
if [ -n "$K" ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$K" > gpurun_out/pytest_sel.log 2>&1
else
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_sel.log 2>&1
fi
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|Error|assert" gpurun_out/pytest_sel.log | tail -40
exit $rc
