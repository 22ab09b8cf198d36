# round 3: A* arena-overflow retry in chunks — exactness tests, 100k route bench, 1M-node scale
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/${TAG:-r3p}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_astar_gpu.py -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u bench/route_bench.py > $O/route_bench.log 2>&1 || { tail -30 $O/route_bench.log; exit 2; }
tail -1 $O/route_bench.log
timeout -k 10 400 python -u bench/astar_scale.py --nodes 1000000 --requests 10000 --radius-km 8 > $O/scale_local.log 2>&1 || { tail -30 $O/scale_local.log; exit 4; }
tail -1 $O/scale_local.log
timeout -k 10 300 python -u bench/astar_scale.py --nodes 1000000 --requests 2000 --radius-km 0 --steps 1 --check 4 > $O/scale_city.log 2>&1 || { tail -30 $O/scale_city.log; exit 5; }
tail -1 $O/scale_city.log
echo done
