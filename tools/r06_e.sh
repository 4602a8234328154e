# Round 6 GPU pass E: blocked Cholesky check, K-shard tests after the shift/ev_used change, emulated rank steps
set -o pipefail
R=$PWD
O=$R/gpurun_out/r06e
mkdir -p $O
timeout -k 10 300 python tools/chol_blk_check.py > $O/chol_blk.jsonl 2> $O/chol_blk.err; echo "chol rc=$?" > $O/rc.txt
timeout -k 10 420 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_kshard_rank.py tests/test_gpu_kshard_native.py > $O/pytest.log 2>&1 || exit 1
for rs in 0 8 16; do
  timeout -k 10 200 python tools/kshard_native_step.py --K 16 --steps 30 --emulate-world 8:0 --reserve $rs > $O/rank16_e8_r$rs.json 2>&1 || exit 1
  QCE_CHOL=blk timeout -k 10 200 python tools/kshard_native_step.py --K 16 --steps 30 --emulate-world 8:0 --reserve $rs > $O/rank16_e8_r${rs}_blk.json 2>&1 || exit 1
done
cd /tmp && export TMPDIR=/tmp
QCE_CHOL=blk timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tr16 -o run --output-format csv -- python3 $R/tools/kshard_native_step.py --K 16 --steps 30 --emulate-world 8:0 --reserve 0 > $O/tr16.json 2> $O/tr16.err || exit 1
cat $O/rc.txt
