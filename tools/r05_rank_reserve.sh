set -o pipefail
mkdir -p gpurun_out/r05r
for r in 0 16; do timeout -k 10 200 python tools/kshard_native_step.py --K 16 --chunks 1 --steps 30 --reserve $r >> gpurun_out/r05r/rank16.jsonl 2>> gpurun_out/r05r/err.txt || exit $?; done
for r in 0 16; do timeout -k 10 200 python tools/kshard_native_step.py --K 32 --N 128 --B 50000 --chunks 1 --steps 20 --reserve $r >> gpurun_out/r05r/rank_cfg4.jsonl 2>> gpurun_out/r05r/err.txt || exit $?; done
timeout -k 10 600 python -u -m pytest tests/test_gpu_kshard_native.py tests/test_gpu_kshard.py tests/test_gpu_f64.py -x -q --timeout 240 --timeout-method thread > gpurun_out/r05r/pytest.log 2>&1
