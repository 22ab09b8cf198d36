# after the batcher queue fix: 2-runner stress (30 rounds), batcher/route-batcher/multirank GPU tests
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r2ay; mkdir -p $O
timeout -k 10 300 python -u tools/stress_batcher_two_runners.py 30 > $O/stress.log 2>&1 || exit 1
timeout -k 10 500 python -u -m pytest tests/test_multirank_gpu.py tests/test_route_batcher_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit 2
echo done
