# round 5: CCH customization time per context (100k and 1M nodes) and PMC of its level kernels
ROOT=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
O=$ROOT/gpurun_out/r5c; mkdir -p $O
timeout -k 10 200 python3 $ROOT/bench/cch_customize_bench.py --contexts 5 --check > $O/cust_100k.jsonl 2>&1 || { tail -20 $O/cust_100k.jsonl; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/stats -o cust --output-format csv -- python3 $ROOT/bench/cch_customize_bench.py --contexts 3 > $O/stats.log 2>&1 || { tail -20 $O/stats.log; exit 2; }
G1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_VALU SQ_INSTS_SALU"
G2="FETCH_SIZE"
G3="WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"
G4="TCC_ATOMIC_sum GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
for G in "$G1" "$G2" "$G3" "$G4"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $G -d $O/pmc$i -o cust --output-format csv -- python3 $ROOT/bench/cch_customize_bench.py --contexts 2 > $O/pmc$i.log 2>&1 || echo "pmc group $i failed rc=$?"
done
timeout -k 10 400 python3 $ROOT/bench/cch_customize_bench.py --nodes 1000000 --contexts 3 > $O/cust_1m.jsonl 2>&1 || { tail -20 $O/cust_1m.jsonl; exit 3; }
echo done
