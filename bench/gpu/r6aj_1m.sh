#!/bin/bash
# 1M-node city: supernodal fronts (default, checked against the CPU reference) vs per-level kernels
set -o pipefail
O=gpurun_out/r6aj; mkdir -p $O
ROUTEST_CCH_DENSE=0 timeout -k 10 300 python -u bench/cch_customize_bench.py --nodes 1000000 --contexts 4 > $O/cust_1m_d0.jsonl 2>&1 || { tail -5 $O/cust_1m_d0.jsonl; exit 1; }
echo "1m d0 $(tail -1 $O/cust_1m_d0.jsonl)"
timeout -k 10 900 python -u bench/cch_customize_bench.py --nodes 1000000 --contexts 4 --check > $O/cust_1m_d8.jsonl 2>&1 || { tail -5 $O/cust_1m_d8.jsonl; exit 1; }
echo "1m d8 $(tail -1 $O/cust_1m_d8.jsonl)"
