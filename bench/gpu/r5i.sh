# round 5: persistence (row texts prepared on the assembly threads, time-ordered row ids) on the
# full bench line; route-service / persistence GPU tests; watchdog rehearsal
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r5i; mkdir -p $O
stop() { rc=$1; [ $rc -eq 124 -o $rc -eq 137 -o $rc -eq 134 -o $rc -eq 139 ] && { echo "GPU step ended rc=$rc: stopping"; exit $rc; }; [ $rc -ne 0 ] && echo "step rc=$rc"; }
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_frontend_gpu.py tests/test_native_server_gpu.py > $O/tests.log 2>&1; stop $?
timeout -k 10 170 python -u -m pytest -x -v -s --timeout 160 --timeout-method thread tests/test_native_lifecycle_gpu.py -k hung > $O/watchdog.log 2>&1; stop $?
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1; stop $?
echo done
