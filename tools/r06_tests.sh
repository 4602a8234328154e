# Round 6: the whole GPU suite on this build, then smoke()
set -o pipefail
R=$PWD
O=$R/gpurun_out/r06t
mkdir -p $O
timeout -k 10 1500 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > $O/gpu_pytest.log 2>&1; echo "pytest rc=$?" > $O/rc.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; echo "smoke rc=$?" >> $O/rc.txt
cat $O/rc.txt
