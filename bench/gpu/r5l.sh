# round 5: a flush over many routing contexts plans in one round trip (plan_multi_road batched over
# groups); column-split training backward (train_bwd_kernel NBW = 1) — gradients vs autograd and vs
# the full-width kernel, then the 64k / 1M training step; routing-context bench again
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r5l; mkdir -p $O
stop() { rc=$1; [ $rc -eq 124 -o $rc -eq 137 -o $rc -eq 134 -o $rc -eq 139 ] && { echo "GPU step ended rc=$rc: stopping"; exit $rc; }; [ $rc -ne 0 ] && echo "step rc=$rc"; }
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_train_gpu.py > $O/train_tests.log 2>&1; stop $?
timeout -k 10 300 python -u bench.py --gcn-steps 0 --route-steps 0 --p50 0 > $O/bench_train.log 2>&1; stop $?
timeout -k 10 240 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_cch_async_gpu.py tests/test_frontend_gpu.py > $O/route_tests.log 2>&1; stop $?
timeout -k 10 400 python -u bench/route_context_bench.py --phases single,cycle64,hour,hour_noprefetch > $O/ctx100k.jsonl 2>$O/ctx100k.err; stop $?
echo done
