# round 3: arena-gated longest-first ordering — A* tests, 100k route step, 1M-node local + city steps
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r3ac; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_astar_gpu.py -m gpu > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 2; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u bench/route_bench.py > $O/rb.log 2>&1 || { tail -20 $O/rb.log; exit 3; }
tail -1 $O/rb.log
timeout -k 10 400 python -u bench/astar_scale.py --nodes 1000000 --requests 10000 --radius-km 8 > $O/scale_local.log 2>&1 || { tail -30 $O/scale_local.log; exit 4; }
tail -1 $O/scale_local.log
timeout -k 10 300 python -u bench/astar_scale.py --nodes 1000000 --requests 2000 --radius-km 0 --steps 1 --check 4 > $O/scale_city.log 2>&1 || { tail -30 $O/scale_city.log; exit 5; }
tail -1 $O/scale_city.log
echo done
