# round 6: route tests again (one non-blocking stream per device for the app's route flushes);
# wgrad256 probe A/B (64x2 / 32x4 vs wgrad<9>) and PMC passes on both dW2 kernels
ROOT=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $ROOT
O=$ROOT/gpurun_out/r6f; mkdir -p $O
stop() { rc=$1; [ $rc -eq 124 -o $rc -eq 137 -o $rc -eq 134 -o $rc -eq 139 ] && { echo "GPU step ended rc=$rc: stopping"; exit $rc; }; [ $rc -ne 0 ] && echo "step rc=$rc"; }
timeout -k 10 120 python -u bench/wgrad_probe.py --iters 20 > $O/probe_64x2.jsonl 2>&1; stop $?
ROUTEST_WGRAD256_CFG=32x4 timeout -k 10 120 python -u bench/wgrad_probe.py --iters 20 --kernels wgrad256 > $O/probe_32x4.jsonl 2>&1; stop $?
cat $O/probe_64x2.jsonl $O/probe_32x4.jsonl
timeout -k 10 200 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_route_batcher_gpu.py > $O/batcher_tests.log 2>&1; stop $?
tail -1 $O/batcher_tests.log
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_native_lifecycle_gpu.py -k "bounded or hung" -s > $O/lifecycle.log 2>&1; stop $?
grep -E "passed|failed" $O/lifecycle.log | tail -1
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_cch_async_gpu.py tests/test_frontend_gpu.py > $O/route_tests.log 2>&1; stop $?
tail -1 $O/route_tests.log
G1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
G2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_LDS_IDX_ACTIVE FETCH_SIZE"
G3="TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum"
i=0
for G in "$G1" "$G2" "$G3"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $G -d $O/pmc_$i -o w --output-format csv -- python3 $ROOT/bench/wgrad_probe.py --iters 5 > $O/pmc_$i.log 2>&1 || { echo "pmc pass $i failed rc=$?"; tail -5 $O/pmc_$i.log; exit 1; }
done
echo pmc done
