set -o pipefail
mkdir -p gpurun_out/r05k
for K in 16; do for c in 1 2; do timeout -k 10 200 python tools/kshard_native_step.py --K $K --chunks $c --steps 30 >> gpurun_out/r05k/rank16.jsonl 2>> gpurun_out/r05k/err.txt || exit $?; done; done
for c in 1 2; do timeout -k 10 200 python tools/kshard_native_step.py --K 32 --N 128 --B 50000 --chunks $c --steps 20 >> gpurun_out/r05k/rank_cfg4.jsonl 2>> gpurun_out/r05k/err.txt || exit $?; done
for cfg in cfg1 cfg2 cfg3 cfg4 cfg5; do timeout -k 10 300 python bench.py --config $cfg --cpu-seconds 0 > gpurun_out/r05k/$cfg.json 2>> gpurun_out/r05k/err.txt || exit $?; done
