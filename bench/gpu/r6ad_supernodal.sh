#!/bin/bash
# supernodal CCH customization: GPU tests, then customize times (default fronts vs per-level)
set -o pipefail
O=gpurun_out/r6ad; mkdir -p $O
timeout -k 10 400 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_cch_gpu.py -k tails > $O/test_cch.log 2>&1 || { tail -30 $O/test_cch.log; exit 1; }
tail -1 $O/test_cch.log
for thr in 8 0 16 32; do
  ROUTEST_CCH_DENSE=$thr timeout -k 10 200 python -u bench/cch_customize_bench.py --nodes 100000 --contexts 6 --check > $O/cust_100k_d$thr.jsonl 2>&1 || { tail -5 $O/cust_100k_d$thr.jsonl; exit 1; }
  tail -1 $O/cust_100k_d$thr.jsonl
done
