set -o pipefail
R=$PWD
mkdir -p gpurun_out/r05s
timeout -k 10 300 python -u -m pytest tests/test_gpu_f64.py -x -q -k "sweep or stream_k or vs_oracle" --timeout 200 --timeout-method thread > gpurun_out/r05s/pytest.log 2>&1 || exit $?
for c in cfg2 cfg1 metric; do timeout -k 10 300 python bench.py --config $c --sweep --steps 10 > gpurun_out/r05s/sweep_$c.json 2>> gpurun_out/r05s/err.txt || exit $?; done
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r05s/prof -o run --output-format csv -- python3 $R/bench.py --config cfg2 --sweep --steps 10 > $R/gpurun_out/r05s/sweep_cfg2_prof.json 2>> $R/gpurun_out/r05s/err.txt
