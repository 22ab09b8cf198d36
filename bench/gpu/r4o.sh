# round 4: group-committed persistence thread + background WAL checkpoints — frontend tests, soak, route HTTP
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
export TMPDIR=/tmp
O=$ROOT/gpurun_out/r4o; mkdir -p $O
timeout -k 10 250 python -u -m pytest tests/test_frontend_gpu.py -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 2; }
tail -1 $O/pytest.log
timeout -k 10 300 python3 tools/app_soak.py --stack --clients 128 --seconds 20 > $O/soak.log 2>&1 || { tail -20 $O/soak.log; exit 5; }
tail -1 $O/soak.log | cut -c1-2500
timeout -k 10 200 python3 bench/route_http_bench.py --provider graph --modes native --seconds 6 --threads 8 --client-threads 8 > $O/http.log 2>&1 || { tail -20 $O/http.log; exit 3; }
tail -3 $O/http.log | cut -c1-2000
