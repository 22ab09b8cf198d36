# round 4: fresh upstream connections after idle — frontend + lifecycle tests, soak
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
export TMPDIR=/tmp
O=$ROOT/gpurun_out/r4r; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_frontend_gpu.py tests/test_native_lifecycle_gpu.py -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 2; }
tail -1 $O/pytest.log
timeout -k 10 300 python3 tools/app_soak.py --stack --clients 128 --seconds 20 > $O/soak.log 2>&1 || { tail -20 $O/soak.log; exit 7; }
tail -1 $O/soak.log | cut -c1-3000
