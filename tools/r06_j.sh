set -o pipefail
R=$PWD
O=$R/gpurun_out/r06j
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tr16 -o run --output-format csv -- python3 $R/tools/kshard_native_step.py --K 16 --steps 30 --emulate-world 8:0 --reserve 0 > $O/tr16.json 2> $O/tr16.err || exit 1
