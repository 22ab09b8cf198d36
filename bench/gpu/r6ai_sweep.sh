#!/bin/bash
# supernodal threshold sweep (ROUTEST_CCH_DENSE) on the 100k graph, then the 1M city (fronts vs per-level)
set -o pipefail
O=gpurun_out/r6ai; mkdir -p $O
for thr in 1 2 4 8 16; do
  ROUTEST_CCH_DENSE=$thr timeout -k 10 200 python -u bench/cch_customize_bench.py --nodes 100000 --contexts 6 --check > $O/cust_100k_d$thr.jsonl 2>&1 || { tail -5 $O/cust_100k_d$thr.jsonl; exit 1; }
  echo "d$thr $(tail -1 $O/cust_100k_d$thr.jsonl)"
done
for thr in 8 0; do
  ROUTEST_CCH_DENSE=$thr timeout -k 10 400 python -u bench/cch_customize_bench.py --nodes 1000000 --contexts 4 --check > $O/cust_1m_d$thr.jsonl 2>&1 || { tail -5 $O/cust_1m_d$thr.jsonl; exit 1; }
  echo "1m d$thr $(tail -1 $O/cust_1m_d$thr.jsonl)"
done
