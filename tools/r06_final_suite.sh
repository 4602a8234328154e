#!/bin/bash
# Round-6 final: the whole GPU suite on this tree's library, then smoke() (outputs under gpurun_out/r06fs/).
set -o pipefail
R=$PWD
O=$R/gpurun_out/r06fs
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > $O/gpu_pytest.log 2>&1 || { tail -40 $O/gpu_pytest.log; exit 1; }
tail -2 $O/gpu_pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
cat $O/smoke.log
