# round 4: route_core put_coord bound — frontend byte-identity tests on the rebuilt route service
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
export TMPDIR=/tmp
O=$ROOT/gpurun_out/r4at; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_frontend_gpu.py tests/test_route_batcher_gpu.py -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 2; }
tail -1 $O/pytest.log
