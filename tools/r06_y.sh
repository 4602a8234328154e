#!/bin/bash
# Round 6: smoke() and the K-shard rank tests on the final tree (build f176c76c32a8d9fe).
set -o pipefail
R=$PWD
O=$R/gpurun_out/r06y
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_kshard_rank.py tests/test_golden_bench_configs.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
