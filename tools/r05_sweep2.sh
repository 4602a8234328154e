set -o pipefail
R=$PWD
mkdir -p gpurun_out/r05s2
for r in 0 16 32 64; do QCE_SWEEP_RESERVE=$r timeout -k 10 300 python bench.py --config cfg2 --sweep --steps 10 --no-parity > gpurun_out/r05s2/sweep_cfg2_r$r.json 2>> gpurun_out/r05s2/err.txt || exit $?; done
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r05s2/prof -o run --output-format csv -- python3 $R/bench.py --config cfg2 --cpu-seconds 0 --no-extras > $R/gpurun_out/r05s2/cfg2_prof.json 2>> $R/gpurun_out/r05s2/err.txt
