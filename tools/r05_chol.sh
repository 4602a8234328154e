set -o pipefail
mkdir -p gpurun_out/r05c
for c in metric cfg2; do for t in 256 512 1024; do QCE_CHOL_THREADS=$t timeout -k 10 120 python tools/prepare_time.py $c >> gpurun_out/r05c/prep.jsonl 2>> gpurun_out/r05c/err.txt || exit $?; done; done
