set -o pipefail
R=$PWD
mkdir -p gpurun_out/r05p
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r05p/k16 -o run --output-format csv -- python3 $R/tools/kshard_native_step.py --K 16 --chunks 1 --steps 30 > $R/gpurun_out/r05p/k16.json 2> $R/gpurun_out/r05p/k16.err
