# A* exact host fallback for overflowed searches: A* tests + route bench (fallback count stays 0)
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r2bg; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_astar_gpu.py tests/test_route_batcher_gpu.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 200 python -u bench/route_bench.py --steps 5 --warmup 1 > $O/route.log 2>&1 || exit 2
echo done
