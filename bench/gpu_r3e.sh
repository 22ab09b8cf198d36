# round 3: full GPU suite + native route benches (both providers) after the adaptive A* stage rule
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r3e; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 400 python -u bench/route_http_bench.py --provider graph > $O/route_graph.log 2>&1 || { tail -40 $O/route_graph.log; exit 3; }
tail -1 $O/route_graph.log
timeout -k 10 300 python -u bench/route_http_bench.py --provider haversine > $O/route_hav.log 2>&1 || { tail -40 $O/route_hav.log; exit 2; }
tail -1 $O/route_hav.log
timeout -k 10 300 python -u tools/app_soak.py --stack --seconds 20 --clients 128 > $O/soak_stack.log 2>&1 || { tail -20 $O/soak_stack.log; exit 4; }
tail -1 $O/soak_stack.log
echo done
