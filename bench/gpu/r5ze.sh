# round 5: builders started with the route service (allocations at startup): route / CCH tests,
# watchdog rehearsal
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r5ze; mkdir -p $O
stop() { rc=$1; [ $rc -eq 124 -o $rc -eq 137 -o $rc -eq 134 -o $rc -eq 139 ] && { echo "GPU step ended rc=$rc: stopping"; exit $rc; }; [ $rc -ne 0 ] && echo "step rc=$rc"; }
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_cch_gpu.py tests/test_cch_async_gpu.py tests/test_frontend_gpu.py tests/test_native_server_gpu.py > $O/tests.log 2>&1; stop $?
tail -1 $O/tests.log
timeout -k 10 170 python -u -m pytest -x -v -s --timeout 160 --timeout-method thread tests/test_native_lifecycle_gpu.py > $O/lifecycle.log 2>&1; stop $?
tail -1 $O/lifecycle.log
