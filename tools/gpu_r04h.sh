#!/bin/bash
# Round 4: the whole GPU suite (one process) and smoke() on the current tree.
set -o pipefail
mkdir -p gpurun_out/r04h
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 170 --timeout-method thread > gpurun_out/r04h/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r04h/pytest.log; grep -E "FAILED|ERROR" gpurun_out/r04h/pytest.log | head -20
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04h/smoke.log 2>&1 || { tail -30 gpurun_out/r04h/smoke.log; exit 1; }
tail -2 gpurun_out/r04h/smoke.log
exit $rc
