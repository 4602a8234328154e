#!/bin/bash
# Device-EM GPU checks (tests/test_fit.py).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/fit; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_fit.py -m gpu -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed|Error|assert" $O/pytest.log | tail -40; exit $rc
