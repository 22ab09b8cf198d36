# round 6: compact route records + bounded failover on the GPU: native-server / frontend / lifecycle
# tests, then the watchdog rehearsal under a HIP runtime + kernel trace (the profiler segfaults in its
# own teardown after writing the CSVs: the CPU-only summary still runs on what it wrote)
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
export TMPDIR=/tmp
O=$ROOT/gpurun_out/r6c; mkdir -p $O
stop() { rc=$1; [ $rc -eq 124 -o $rc -eq 137 -o $rc -eq 134 -o $rc -eq 139 ] && { echo "GPU step ended rc=$rc: stopping"; exit $rc; }; [ $rc -ne 0 ] && echo "step rc=$rc"; }
( while sleep 30; do echo "tick $(date +%T)"; done ) & TICK=$!
timeout -k 10 500 python -u -m pytest -v --timeout 240 --timeout-method thread tests/test_frontend_gpu.py tests/test_native_server_gpu.py tests/test_native_lifecycle_gpu.py > $O/tests.log 2>&1; stop $?
tail -3 $O/tests.log
grep -E "PASS|FAIL|ERROR" $O/tests.log | grep -v "^tests.*PASSED" | head -20
export GPU_MAX_HW_QUEUES=32 ROUTEST_GPU_DEADLINE_MS=100 ROUTEST_ROUTE_DEADLINE_MS=300 ROUTEST_PERSIST_IDLE_MS=0 ROUTEST_QUARANTINE_PROBE_MS=60000 ROUTEST_HANG_ARM=1
timeout -k 10 300 rocprofv3 --hip-runtime-trace --kernel-trace --output-format csv -d /tmp/wd -- python3 -u tests/_watchdog_child.py > $O/child_traced.log 2>&1
echo "traced rc=$?"
ls -la /tmp/wd/*/
timeout -k 10 240 python3 tools/slow_calls.py /tmp/wd 50 > $O/slow_calls.txt 2>&1
echo "summary rc=$?"
head -60 $O/slow_calls.txt
kill $TICK
