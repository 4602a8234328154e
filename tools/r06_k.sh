set -o pipefail
R=$PWD
O=$R/gpurun_out/r06k
mkdir -p $O
for rep in 1 2; do for pr in 0 1; do
  QCE_KSHARD_PRIO=$pr timeout -k 10 200 python tools/kshard_native_step.py --K 16 --steps 40 --emulate-world 8:0 --reserve 0 --no-parity > $O/rank16_p${pr}_$rep.json 2>&1 || exit 1
done; done
cd /tmp && export TMPDIR=/tmp
QCE_KSHARD_PRIO=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr16 -o run --output-format csv -- python3 $R/tools/kshard_native_step.py --K 16 --steps 30 --emulate-world 8:0 --reserve 0 --no-parity > $O/tr16.json 2> $O/tr16.err || exit 1
