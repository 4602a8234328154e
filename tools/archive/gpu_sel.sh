#!/bin/bash
# Selected GPU test files (SEL), one process.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/sel; mkdir -p $O
timeout -k 10 400 python -u -m pytest $SEL -m gpu -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; grep -E "PASSED|FAILED|passed|failed|Error" $O/pytest.log | tail -20; exit $rc
