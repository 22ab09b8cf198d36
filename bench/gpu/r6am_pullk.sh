#!/bin/bash
# below-front pull: wave kernel for levels with a >= 64-arc node (default) vs the lane/wave mean-degree rule only
O=gpurun_out/r6am; mkdir -p $O
for k in 64 1000000 64 1000000; do
  ROUTEST_CCH_PULL_WAVE_K=$k timeout -k 10 200 python -u bench/cch_customize_bench.py --nodes 100000 --contexts 6 > $O/cust_wk$k.jsonl 2>&1 || exit 1
  echo "wave_k=$k $(tail -1 $O/cust_wk$k.jsonl | cut -c90-200)"
done
