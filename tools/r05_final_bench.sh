set -o pipefail
R=$PWD
mkdir -p gpurun_out/r05f
timeout -k 10 300 python bench.py > gpurun_out/r05f/metric_bench.json 2> gpurun_out/r05f/metric_bench.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r05f/prof -o run --output-format csv -- python3 $R/bench.py > $R/gpurun_out/r05f/metric_bench_prof.json 2> $R/gpurun_out/r05f/metric_bench_prof.err || exit $?
cd $R && timeout -k 10 200 python bench.py --dropin --no-extras --cpu-seconds 0 --steps 5 > gpurun_out/r05f/dropin_bench.json 2> gpurun_out/r05f/dropin.err
