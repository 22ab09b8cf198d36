# round 4: frontend + observed-GCN GPU tests, 1M-node city-wide CCH, soak, GCN bench, bench.py
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
export TMPDIR=/tmp
O=$ROOT/gpurun_out/r4j; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_frontend_gpu.py tests/test_gcn_observed.py -x -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 3; }
tail -1 $O/pytest.log
timeout -k 10 500 python3 bench/astar_scale.py --engine cch --nodes 1000000 --requests 2000 --radius-km 0 --steps 3 > $O/scale_1m.log 2>&1 || { tail -20 $O/scale_1m.log; exit 4; }
tail -1 $O/scale_1m.log
timeout -k 10 300 python3 tools/app_soak.py --stack --clients 128 --seconds 20 > $O/soak.log 2>&1 || { tail -20 $O/soak.log; exit 5; }
tail -1 $O/soak.log | cut -c1-2000
timeout -k 10 400 python3 bench/gcn_observed_bench.py --nodes 100000 --trips 50000 --steps 600 --lr 1e-2 > $O/gcn_observed.log 2>&1 || { tail -20 $O/gcn_observed.log; exit 6; }
tail -1 $O/gcn_observed.log
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 7; }
tail -1 $O/bench.log
