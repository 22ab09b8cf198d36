# round 3: full GPU suite + smoke + headline bench after the A* ordering / length split; A* at 1M nodes
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r3z; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 2; }
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 3; }
tail -1 $O/bench.log
timeout -k 10 400 python -u bench/astar_scale.py --nodes 1000000 --requests 10000 --radius-km 8 > $O/scale_local.log 2>&1 || { tail -30 $O/scale_local.log; exit 4; }
tail -1 $O/scale_local.log
timeout -k 10 300 python -u bench/astar_scale.py --nodes 1000000 --requests 2000 --radius-km 0 --steps 1 --check 4 > $O/scale_city.log 2>&1 || { tail -30 $O/scale_city.log; exit 5; }
tail -1 $O/scale_city.log
echo done
