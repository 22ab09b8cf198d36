#!/bin/bash
# whole GPU suite with the per-level CCH (ROUTEST_CCH_DENSE=0): is the watchdog test's failure the fronts'?
ROOT=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $ROOT
O=$ROOT/gpurun_out/r6at; mkdir -p $O
ROUTEST_CCH_DENSE=0 timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_suite_d0.log 2>&1
rc=$?
tail -3 $O/gpu_suite_d0.log
exit $rc
