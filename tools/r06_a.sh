# Round 6 GPU pass A: K-shard rank / lifecycle tests, the emulated world-8 rank step (metric K=16, cfg4 K=32),
# a kernel trace of the metric rank, the exit-time teardown under rocprofv3 (with and without the atexit close),
# and the cfg4 bench line on the new 3M halves kernel -- VERDICT r5 #1, #2, #4.
set -o pipefail
R=$PWD
O=$R/gpurun_out/r06a
mkdir -p $O
timeout -k 10 420 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_kshard_rank.py tests/test_gpu_kshard_native.py > $O/pytest.log 2>&1 || exit 1
for rs in 16 8 0; do
  timeout -k 10 200 python tools/kshard_native_step.py --K 16 --steps 30 --emulate-world 8:0 --reserve $rs > $O/rank16_e8_r$rs.json 2>&1 || exit 1
done
timeout -k 10 200 python tools/kshard_native_step.py --K 16 --steps 30 --reserve 16 > $O/rank16_w1_r16.json 2>&1 || exit 1
timeout -k 10 200 python tools/kshard_native_step.py --K 32 --N 128 --B 50000 --steps 10 --emulate-world 8:0 > $O/rank32_cfg4_e8.json 2>&1 || exit 1
timeout -k 10 300 python bench.py --config cfg4 --steps 10 --warmup 2 --cpu-seconds 0 > $O/cfg4_bench.json 2> $O/cfg4_bench.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tr16 -o run --output-format csv -- python3 $R/tools/kshard_native_step.py --K 16 --steps 30 --emulate-world 8:0 > $O/tr16.json 2> $O/tr16.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/noclose -o run --output-format csv -- python3 $R/tools/kshard_native_step.py --K 16 --steps 5 --no-close --no-parity > $O/noclose.json 2> $O/noclose.err; echo "noclose rc=$?" >> $O/rc.txt
QCE_NO_EXIT_CLOSE=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $O/noexit -o run --output-format csv -- python3 $R/tools/kshard_native_step.py --K 16 --steps 5 --no-close --no-parity > $O/noexit.json 2> $O/noexit.err; echo "noexit rc=$?" >> $O/rc.txt
cat $O/rc.txt
