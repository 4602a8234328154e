set -o pipefail
O=$PWD/gpurun_out/r06d
mkdir -p $O
rm -f $O/overlap2.jsonl
for cfg in "240 256 256 1" "240 16 256 1" "248 256 256 1" "224 256 256 1" "256 256 256 1" "240 256 256 0"; do
  timeout -k 10 60 tools/probe/overlap_probe $cfg >> $O/overlap2.jsonl 2>> $O/overlap2.err || exit 1
done
