# Round 6 GPU pass G: prefetched filter kernel (prepare time, tables), rank step, cfg4 prefetch-distance A/B
set -o pipefail
R=$PWD
O=$R/gpurun_out/r06g
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_kshard_rank.py > $O/pytest.log 2>&1 || exit 1
for c in metric cfg2 cfg1; do timeout -k 10 120 python tools/prepare_time.py $c >> $O/prepare.jsonl 2>> $O/prepare.err || exit 1; done
timeout -k 10 200 python tools/kshard_native_step.py --K 16 --steps 30 --emulate-world 8:0 --reserve 0 > $O/rank16_e8_r0.json 2>&1 || exit 1
L=quantized_channel_estimation_amd
timeout -k 10 600 python tools/lib_ab.py --config cfg4 --rounds 2 main:$L/libqce.so eh2:$L/libqce_eh2.so eh6:$L/libqce_eh6.so > $O/cfg4_ab.jsonl 2> $O/cfg4_ab.err || exit 1
