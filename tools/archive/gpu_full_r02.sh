#!/bin/bash
# Full GPU suite + smoke (round-end rehearsal); logs under gpurun_out/full.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/full; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; grep -E "FAILED|Error" $O/pytest.log | head -5; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
