# round 5 (late): multi-GPU readiness rehearsal again with the round-end code (every rank on GPU 0):
# tests/test_multigpu.py and bench.py --gpus 2 and --gpus 4; the watchdog rehearsal
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r5x; mkdir -p $O
stop() { rc=$1; [ $rc -eq 124 -o $rc -eq 137 -o $rc -eq 134 -o $rc -eq 139 ] && { echo "GPU step ended rc=$rc: stopping"; exit $rc; }; [ $rc -ne 0 ] && echo "step rc=$rc"; }
timeout -k 10 500 env ROUTEST_TEST_SHARE_GPU=1 python -u -m pytest -x -v --timeout 450 --timeout-method thread tests/test_multigpu.py > $O/multigpu_share.log 2>&1; stop $?
timeout -k 10 300 env ROUTEST_BENCH_SHARE_GPU=1 python bench.py --gpus 2 --steps 10 --warmup 3 --p50 0 > $O/bench_share2.log 2>&1; stop $?
timeout -k 10 300 env ROUTEST_BENCH_SHARE_GPU=1 python bench.py --gpus 4 --steps 10 --warmup 3 --p50 0 > $O/bench_share4.log 2>&1; stop $?
timeout -k 10 170 python -u -m pytest -x -v -s --timeout 160 --timeout-method thread tests/test_native_lifecycle_gpu.py -k hung > $O/watchdog.log 2>&1; stop $?

timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_cch_gpu.py tests/test_cch_async_gpu.py > $O/cch_tests.log 2>&1; stop $?
timeout -k 10 240 python -u bench/route_context_bench.py --nodes 1000000 --concurrency 256 --phases fresh > $O/fresh_default.jsonl 2>$O/fresh_default.err; stop $?
echo done2
