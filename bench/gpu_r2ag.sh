# auto variant 20: kernel tests + smoke + default bench
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r2ag; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_eta_kernel_gpu.py tests/test_native_server_gpu.py tests/test_bench_contract_gpu.py -x -q --timeout 250 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 240 python -u -c "import __graft_entry__ as e; e.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 2
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 3
echo done
