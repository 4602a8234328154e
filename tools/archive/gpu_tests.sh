#!/bin/bash
# Whole GPU test suite, one process.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/tests; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed|Error" $O/pytest.log | tail -30; exit $rc
