# bench.py contract tests after the one-shot fallback edit
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r2bj; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_bench_contract_gpu.py -x -v --timeout 250 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
echo done
