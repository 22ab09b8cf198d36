# round 3: pipelined route service — front-end tests + graph/haversine route bench with stage times
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r3c; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_frontend_gpu.py -x -q --timeout 240 --timeout-method thread > $O/pytest_front.log 2>&1 || { tail -80 $O/pytest_front.log; exit 1; }
tail -3 $O/pytest_front.log
timeout -k 10 400 python -u bench/route_http_bench.py --provider graph --modes native > $O/route_graph.log 2>&1 || { tail -40 $O/route_graph.log; exit 3; }
tail -2 $O/route_graph.log
timeout -k 10 300 python -u bench/route_http_bench.py --provider haversine --modes native > $O/route_hav.log 2>&1 || { tail -40 $O/route_hav.log; exit 2; }
tail -2 $O/route_hav.log
echo done
