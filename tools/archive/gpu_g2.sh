#!/bin/bash
# Selected GPU tests ($SEL), then the Fourier-kernel PMC passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/g2; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$SEL" > $O/pytest.log 2>&1
rc=$?; grep -E "passed|failed|Error|assert" $O/pytest.log | tail -5; [ $rc -ne 0 ] && exit $rc
bash tools/pmc_fft.sh
