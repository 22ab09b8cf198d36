# round 3: sparse-state tiered A* — exactness tests, graph-route tests, 1M-node scale, 100k legs/s
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r3f; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_multirank_gpu.py tests/test_comm_gpu.py -x -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python -u bench/route_bench.py > $O/route_bench.log 2>&1 || { tail -30 $O/route_bench.log; exit 2; }
tail -2 $O/route_bench.log
timeout -k 10 300 python -u bench/astar_tail.py > $O/astar_tail.log 2>&1 || { tail -30 $O/astar_tail.log; exit 3; }
tail -3 $O/astar_tail.log
timeout -k 10 400 python -u bench/astar_scale.py --nodes 1000000 --requests 10000 --radius-km 8 > $O/scale_local.log 2>&1 || { tail -30 $O/scale_local.log; exit 4; }
tail -1 $O/scale_local.log
timeout -k 10 400 python -u bench/astar_scale.py --nodes 1000000 --requests 10000 --radius-km 0 --steps 1 > $O/scale_city.log 2>&1 || { tail -30 $O/scale_city.log; exit 5; }
tail -1 $O/scale_city.log
timeout -k 10 400 python -u bench/route_http_bench.py --provider graph > $O/route_graph.log 2>&1 || { tail -40 $O/route_graph.log; exit 6; }
tail -1 $O/route_graph.log
echo done
