#!/bin/bash
# whole GPU suite + smoke with the supernodal CCH default
ROOT=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $ROOT
O=$ROOT/gpurun_out/${OUT:-r6ak}; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1
rc=$?
tail -3 $O/gpu_suite.log
if [ $rc -eq 124 -o $rc -eq 137 -o $rc -eq 134 -o $rc -eq 139 ]; then exit $rc; fi
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1; echo "smoke rc=$?"; tail -1 $O/smoke.log
exit $rc
