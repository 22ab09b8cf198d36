#!/bin/bash
# whole GPU suite with the watchdog rehearsal hoisted to the front of the session (run_first)
ROOT=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $ROOT
O=$ROOT/gpurun_out/r6av; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_suite.log 2>&1
rc=$?
tail -3 $O/gpu_suite.log
exit $rc
