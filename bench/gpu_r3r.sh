# round 3: headline bench after the A* tiering change + route/A* GPU tests
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r3r; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_astar_gpu.py tests/test_route_kernels_gpu.py tests/test_route_batcher_gpu.py tests/test_train_gpu.py -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 3; }
tail -1 $O/bench.log
echo done
