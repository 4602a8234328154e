set -o pipefail
R=$PWD
O=$R/gpurun_out/r06b
mkdir -p $O
timeout -k 10 120 python tools/rs_tail_probe.py > $O/rs_probe.jsonl 2> $O/rs_probe.err || exit 1
