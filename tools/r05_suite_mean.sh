set -o pipefail
mkdir -p gpurun_out/r05m
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_gpu_suite2.log 2>&1 || exit $?
for c in cfg3 cfg5; do timeout -k 10 200 python bench.py --config $c --mean --cpu-seconds 0 > gpurun_out/r05m/${c}_mean.json 2>> gpurun_out/r05m/err.txt || exit $?; done
