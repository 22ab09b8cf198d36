# round 3 final check: bench.py with the 98304-slot route step + bench contract / routing GPU tests
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r3ak; mkdir -p $O
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 3; }
tail -1 $O/bench.log
timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_bench_contract_gpu.py tests/test_route_batcher_gpu.py -m gpu > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 2; }
tail -1 $O/pytest.log
echo done
