#!/bin/bash
# Round-end check of the committed tree: the whole GPU suite and smoke().
set -o pipefail
mkdir -p gpurun_out/r03s
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r03s/pytest.log 2>&1 || { tail -30 gpurun_out/r03s/pytest.log; exit 1; }
tail -2 gpurun_out/r03s/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03s/smoke.log 2>&1 || { tail -30 gpurun_out/r03s/smoke.log; exit 1; }
tail -2 gpurun_out/r03s/smoke.log
