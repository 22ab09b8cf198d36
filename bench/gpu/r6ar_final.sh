#!/bin/bash
# final-code check: whole GPU suite + smoke, then the 1M city against the CPU reference
ROOT=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $ROOT
O=$ROOT/gpurun_out/r6ar; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1
rc=$?
tail -3 $O/gpu_suite.log
if [ $rc -eq 124 -o $rc -eq 137 -o $rc -eq 134 -o $rc -eq 139 ]; then exit $rc; fi
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1; echo "smoke rc=$?"; tail -1 $O/smoke.log
timeout -k 10 600 python -u bench/cch_customize_bench.py --nodes 1000000 --contexts 4 --check > $O/cust_1m.jsonl 2>&1; echo "1m rc=$? $(tail -1 $O/cust_1m.jsonl)"
exit $rc
