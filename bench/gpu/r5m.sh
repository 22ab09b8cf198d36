# round 5: one launch sequence per flush over all its routing contexts (CCH multi-metric views);
# route byte-identity tests, routing-context bench, full bench line
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r5m; mkdir -p $O
stop() { rc=$1; [ $rc -eq 124 -o $rc -eq 137 -o $rc -eq 134 -o $rc -eq 139 ] && { echo "GPU step ended rc=$rc: stopping"; exit $rc; }; [ $rc -ne 0 ] && echo "step rc=$rc"; }
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_cch_gpu.py tests/test_cch_async_gpu.py tests/test_frontend_gpu.py tests/test_native_server_gpu.py tests/test_history_native_cpu.py > $O/route_tests.log 2>&1; stop $?
timeout -k 10 400 python -u bench/route_context_bench.py --phases single,cycle64,hour,hour_noprefetch > $O/ctx100k.jsonl 2>$O/ctx100k.err; stop $?
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1; stop $?
echo done
