set -o pipefail
O=$PWD/gpurun_out/r06c
mkdir -p $O
timeout -k 10 200 python tools/rs_tail_probe.py 325520 325504 325632 325376 325248 325184 325152 325136 1625000 1625024 1630720 65536 65546 32768 32778 16384 16394 8192 8202 4096 4106 > $O/rs_probe2.jsonl 2> $O/rs_probe2.err || exit 1
