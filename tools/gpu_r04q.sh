#!/bin/bash
# Round 4, final build: the drop-in (numpy host I/O) side line of the metric config (bench.py --dropin).
set -o pipefail
O=gpurun_out/r04q
mkdir -p $O
timeout -k 10 400 python -u bench.py --cpu-seconds 0 --dropin > $O/dropin.json 2> $O/dropin.err || { tail -20 $O/dropin.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/dropin.json'));print(d['value'], d['ms_per_step'], json.dumps(d.get('dropin')))"
