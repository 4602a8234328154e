# Round 6 GPU pass F: the fused prepare (Cy in the gain kernel, V / W in one kernel): tables and parity, prepare time,
# the emulated rank step, cfg1 / cfg2 bench lines
set -o pipefail
R=$PWD
O=$R/gpurun_out/r06f
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_f64.py tests/test_golden_bench_configs.py tests/test_quirks.py tests/test_gpu_kshard_rank.py > $O/pytest.log 2>&1 || exit 1
for c in metric cfg2 cfg1; do timeout -k 10 120 python tools/prepare_time.py $c >> $O/prepare.jsonl 2>> $O/prepare.err || exit 1; done
for rs in 0 8; do
  timeout -k 10 200 python tools/kshard_native_step.py --K 16 --steps 30 --emulate-world 8:0 --reserve $rs > $O/rank16_e8_r$rs.json 2>&1 || exit 1
done
timeout -k 10 200 python tools/kshard_native_step.py --K 32 --N 128 --B 50000 --steps 10 --emulate-world 8:0 --reserve 0 > $O/rank32_cfg4_e8_r0.json 2>&1 || exit 1
for c in cfg1 cfg2; do timeout -k 10 200 python bench.py --config $c --steps 20 --warmup 3 --cpu-seconds 0 > $O/${c}_bench.json 2> $O/${c}_bench.err || exit 1; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tr16 -o run --output-format csv -- python3 $R/tools/kshard_native_step.py --K 16 --steps 30 --emulate-world 8:0 --reserve 0 > $O/tr16.json 2> $O/tr16.err || exit 1
