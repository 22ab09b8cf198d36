# optimizer on the request path: GPU route batcher tests + HTTP req/s bench (haversine, graph)
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=gpurun_out/r2d; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_route_batcher_gpu.py tests/test_astar_gpu.py tests/test_route_kernels_gpu.py -x -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python -u bench/route_http_bench.py --provider haversine --concurrency 2000 > $O/route_http_haversine.log 2>&1 || exit 2
timeout -k 10 400 python -u bench/route_http_bench.py --provider graph --concurrency 1000 > $O/route_http_graph.log 2>&1 || exit 3
echo done
