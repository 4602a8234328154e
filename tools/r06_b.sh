set -o pipefail
R=$PWD
O=$R/gpurun_out/r06b
mkdir -p $O
timeout -k 10 120 python tools/rs_tail_probe.py > $O/rs_probe.jsonl 2> $O/rs_probe.err || exit 1
timeout -k 10 400 python -u -m pytest -v --timeout 150 --timeout-method thread tests/test_gpu_kshard_rank.py > $O/pytest_rank.log 2>&1; echo "rank rc=$?" > $O/rc.txt
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_f64.py -k "3m_matches or f64h" > $O/pytest_f64h.log 2>&1; echo "f64h rc=$?" >> $O/rc.txt
cat $O/rc.txt
