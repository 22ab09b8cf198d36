# round 5: the rest of the GPU suite (serving, routing, bench contract)
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r5h; mkdir -p $O
stop() { rc=$1; [ $rc -eq 124 -o $rc -eq 137 -o $rc -eq 134 -o $rc -eq 139 ] && { echo "GPU step ended rc=$rc: stopping"; exit $rc; }; [ $rc -ne 0 ] && echo "step rc=$rc"; }
timeout -k 10 900 python -u -m pytest -v -m gpu --timeout 300 --timeout-method thread tests/test_cch_gpu.py tests/test_cch_async_gpu.py tests/test_frontend_gpu.py tests/test_native_server_gpu.py tests/test_native_lifecycle_gpu.py tests/test_route_batcher_gpu.py tests/test_bench_contract_gpu.py tests/test_multigpu.py > $O/suite_b.log 2>&1; stop $?
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1; stop $?
echo done
