# round 5: customization with task-table basic + MLP-unrolled perfect pull + wave prune (100k, 1M),
# bit-identity, kernel stats + PMC; latency-watchdog rehearsal after the deferred-free change
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r5e; mkdir -p $O
stop() { rc=$1; [ $rc -eq 124 -o $rc -eq 137 -o $rc -eq 134 -o $rc -eq 139 ] && { echo "GPU step ended rc=$rc: stopping"; exit $rc; }; [ $rc -ne 0 ] && echo "step rc=$rc"; }
timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_cch_gpu.py > $O/test_cch_gpu.log 2>&1; stop $?
timeout -k 10 200 python3 bench/cch_customize_bench.py --contexts 4 --check > $O/cust_100k.jsonl 2>&1; stop $?
timeout -k 10 170 python3 bench/cch_customize_bench.py --nodes 1000000 --contexts 3 > $O/cust_1m.jsonl 2>&1; stop $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 170 rocprofv3 --kernel-trace --stats -d $O/stats -o cust --output-format csv -- python3 $ROOT/bench/cch_customize_bench.py --contexts 3 > $O/stats.log 2>&1; stop $?
G1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_VALU SQ_INSTS_SALU"
G2="FETCH_SIZE"
G3="WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"
i=0
for G in "$G1" "$G2" "$G3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $G -d $O/pmc$i -o cust --output-format csv -- python3 $ROOT/bench/cch_customize_bench.py --contexts 2 > $O/pmc$i.log 2>&1; stop $?
done
cd $ROOT
timeout -k 10 170 python -u -m pytest -x -v -s --timeout 160 --timeout-method thread tests/test_native_lifecycle_gpu.py -k hung > $O/watchdog.log 2>&1; stop $?
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1; stop $?
echo done
