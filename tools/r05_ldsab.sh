#!/bin/bash
# LDS bank-conflict pass (rocprofv3 --pmc, one counter group) of the cfg3 / cfg5 Fourier kernels, zero-mean and
# with means, each under its own time limit; summaries printed from run_counter_collection.csv.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/ldsab
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for c in "cfg3 " "cfg3 --mean" "cfg5 " "cfg5 --mean"; do
  set -- $c
  name=$1${2:+_mean}
  timeout -k 10 -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $OUT/$name -o run --output-format csv -- python3 $R/bench.py --config $1 $2 --steps 2 --warmup 1 --cpu-seconds 0 --no-parity --no-extras > $OUT/$name.log 2>&1 || exit $?
  python3 - $OUT/$name/run_counter_collection.csv $name <<'PY'
import csv, sys, collections
v = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    if r["Kernel_Name"].find("k_fft") < 0:
        continue
    v[r["Kernel_Name"].split("(")[0][-60:]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in v.items():
    bc, act = sum(d["SQ_LDS_BANK_CONFLICT"]), sum(d["SQ_LDS_IDX_ACTIVE"])
    print(sys.argv[2], k, "bank conflicts / LDS active %.4f" % (bc / max(act, 1)))
PY
done
