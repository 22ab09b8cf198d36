#!/bin/bash
# supernodal CCH v2 (1024-thread panel/solve/kk, gather-side finalization): bit-identity test, times, kernel profile
set -o pipefail
O=gpurun_out/${OUT:-r6af}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_cch_gpu.py -k "supernodal or legs_exact" > $O/test_cch.log 2>&1 || { tail -30 $O/test_cch.log; exit 1; }
tail -1 $O/test_cch.log
timeout -k 10 200 python -u bench/cch_customize_bench.py --nodes 100000 --contexts 6 --check > $O/cust_100k.jsonl 2>&1 || { tail -5 $O/cust_100k.jsonl; exit 1; }
tail -1 $O/cust_100k.jsonl
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench/cch_customize_bench.py --nodes 100000 --contexts 3 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
