set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/big
timeout -k 10 300 python -u bench.py --config cfg4 --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/big/cfg4.json 2> gpurun_out/big/cfg4.err || exit $?
cat gpurun_out/big/cfg4.json
timeout -k 10 300 python -u bench.py --config cfg5dense --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/big/cfg5.json 2> gpurun_out/big/cfg5.err || exit $?
cat gpurun_out/big/cfg5.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/big/prof4 -o run --output-format csv -- python -u $GRAFT_REPO_ROOT/bench.py --config cfg4 --steps 3 --warmup 1 --cpu-seconds 0 --no-parity > /dev/null 2>&1 || exit $?
head -12 $GRAFT_REPO_ROOT/gpurun_out/big/prof4/run_kernel_stats.csv | cut -c1-200
