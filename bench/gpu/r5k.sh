# round 5: routing contexts under load (verdict r4 item 2 "done when"): 64 cycling contexts vs one,
# an hour boundary with and without prefetch (100k graph), a fresh context on the 1M city; host
# costs made by the customization; async-context GPU tests
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r5k; mkdir -p $O
stop() { rc=$1; [ $rc -eq 124 -o $rc -eq 137 -o $rc -eq 134 -o $rc -eq 139 ] && { echo "GPU step ended rc=$rc: stopping"; exit $rc; }; [ $rc -ne 0 ] && echo "step rc=$rc"; }
timeout -k 10 240 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_cch_async_gpu.py tests/test_cch_gpu.py > $O/tests.log 2>&1; stop $?
timeout -k 10 400 python -u bench/route_context_bench.py --phases single,cycle64,hour,hour_noprefetch > $O/ctx100k.jsonl 2>$O/ctx100k.err; stop $?
timeout -k 10 300 python -u bench/route_context_bench.py --nodes 1000000 --concurrency 256 --phases fresh > $O/ctx1m.jsonl 2>$O/ctx1m.err; stop $?
echo done
