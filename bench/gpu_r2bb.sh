# route batcher: two workers on one GPU (lock around the shared A* workspace, deadline-polling queue)
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r2bb; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_route_batcher_gpu.py -x -v --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
echo done
