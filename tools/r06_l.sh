# Round 6 GPU pass L: next-tile y prefetch in the headline kernel: parity, metric / K=16 A/B, rank step
set -o pipefail
R=$PWD
O=$R/gpurun_out/r06l
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_fullbatch.py tests/test_gpu_argmax_metric.py tests/test_gpu_f64.py tests/test_gpu_kshard_rank.py > $O/pytest.log 2>&1 || exit 1
L=quantized_channel_estimation_amd
timeout -k 10 500 python tools/lib_ab.py --config metric --rounds 3 main:$L/libqce.so nopre:$L/libqce_nopre.so > $O/metric_ab.jsonl 2> $O/metric_ab.err || exit 1
timeout -k 10 500 python tools/lib_ab.py --config metric --components 16 --rounds 3 main:$L/libqce.so nopre:$L/libqce_nopre.so > $O/k16_ab.jsonl 2> $O/k16_ab.err || exit 1
for v in main nopre; do
  lib=$L/libqce.so; [ $v = nopre ] && lib=$L/libqce_nopre.so
  QCE_LIB=$R/$lib timeout -k 10 200 python tools/kshard_native_step.py --K 16 --steps 40 --emulate-world 8:0 --reserve 0 --no-parity > $O/rank16_$v.json 2>&1 || exit 1
done
