#!/bin/bash
# New GPU tests of this round (FP64 selective modes, quirks, BASELINE configs at full K).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02b; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_f64.py tests/test_quirks.py tests/test_gpu_configs.py -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed|Error|assert" $O/pytest.log | tail -30
exit $rc
