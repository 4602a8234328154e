# Round 6 GPU pass I: the uniform-stream padded-128 3M kernel: parity, cfg4 A/B over the prefetch distance
set -o pipefail
R=$PWD
O=$R/gpurun_out/r06i
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_f64.py -k "3m_matches or f64h" > $O/pytest.log 2>&1 || exit 1
L=quantized_channel_estimation_amd
timeout -k 10 600 python tools/lib_ab.py --config cfg4 --rounds 2 main:$L/libqce.so eh2:$L/libqce_eh2.so eh6:$L/libqce_eh6.so > $O/cfg4_ab.jsonl 2> $O/cfg4_ab.err || exit 1
timeout -k 10 600 python tools/lib_ab.py --config cfg4 --mean --rounds 1 main:$L/libqce.so > $O/cfg4_mean_ab.jsonl 2> $O/cfg4_mean_ab.err || exit 1
