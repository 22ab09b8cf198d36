# round 5: finished route jobs handed back to the reactors in batches: route tests, watchdog, bench line

ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r5zj; mkdir -p $O
stop() { rc=$1; [ $rc -eq 124 -o $rc -eq 137 -o $rc -eq 134 -o $rc -eq 139 ] && { echo "GPU step ended rc=$rc: stopping"; exit $rc; }; [ $rc -ne 0 ] && echo "step rc=$rc"; }
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_frontend_gpu.py tests/test_native_server_gpu.py tests/test_history_native_cpu.py tests/test_cch_async_gpu.py > $O/tests.log 2>&1; stop $?
tail -1 $O/tests.log
timeout -k 10 170 python -u -m pytest -x -q -s --timeout 160 --timeout-method thread tests/test_native_lifecycle_gpu.py -k hung > $O/watchdog.log 2>&1; stop $?
tail -1 $O/watchdog.log
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1; stop $?
echo done
