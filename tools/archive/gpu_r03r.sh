#!/bin/bash
# K-shard with the 2-chunk default: the GPU K-shard tests and a 2-rank gloo rehearsal of the bench on one GPU.
set -o pipefail
mkdir -p gpurun_out/r03r
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kshard.py > gpurun_out/r03r/pytest.log 2>&1 || { tail -30 gpurun_out/r03r/pytest.log; exit 1; }
tail -2 gpurun_out/r03r/pytest.log
timeout -k 10 300 python -u bench.py --gpus 2 --backend gloo --steps 10 --warmup 3 --cpu-seconds 0 --no-extras > gpurun_out/r03r/kshard2_gloo.json 2> gpurun_out/r03r/kshard2_gloo.err || { tail -30 gpurun_out/r03r/kshard2_gloo.err; exit 1; }
cat gpurun_out/r03r/kshard2_gloo.json
