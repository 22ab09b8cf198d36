# round 5: three concurrent context builders (own temporaries each) on a quarter of the CUs; a
# fresh context on the 1M city under load, 64 cold contexts on the 100k graph, sync customization
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r5n; mkdir -p $O
stop() { rc=$1; [ $rc -eq 124 -o $rc -eq 137 -o $rc -eq 134 -o $rc -eq 139 ] && { echo "GPU step ended rc=$rc: stopping"; exit $rc; }; [ $rc -ne 0 ] && echo "step rc=$rc"; }
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_cch_gpu.py tests/test_cch_async_gpu.py tests/test_frontend_gpu.py > $O/route_tests.log 2>&1; stop $?
timeout -k 10 300 python -u bench/route_context_bench.py --phases single,cycle64 > $O/ctx100k.jsonl 2>$O/ctx100k.err; stop $?
timeout -k 10 300 python -u bench/route_context_bench.py --nodes 1000000 --concurrency 256 --phases fresh > $O/ctx1m.jsonl 2>$O/ctx1m.err; stop $?
timeout -k 10 200 python -u bench/cch_customize_bench.py --contexts 6 > $O/cust100k.jsonl 2>&1; stop $?
echo done
