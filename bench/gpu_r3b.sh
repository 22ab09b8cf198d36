# round 3: native front end + route service — GPU tests, then the route HTTP bench (both providers)
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r3b; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_frontend_gpu.py -x -v --timeout 240 --timeout-method thread > $O/pytest_front.log 2>&1 || { tail -80 $O/pytest_front.log; exit 1; }
tail -15 $O/pytest_front.log
timeout -k 10 300 python -u bench/route_http_bench.py --provider haversine --modes native,per_request,batched > $O/route_hav.log 2>&1 || { tail -40 $O/route_hav.log; exit 2; }
tail -5 $O/route_hav.log
timeout -k 10 400 python -u bench/route_http_bench.py --provider graph --modes native > $O/route_graph.log 2>&1 || { tail -40 $O/route_graph.log; exit 3; }
tail -3 $O/route_graph.log
echo done
