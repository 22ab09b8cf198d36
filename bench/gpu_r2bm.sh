# final: bench.py contract tests + default bench line with the calibration ratio keys
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r2bm; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_bench_contract_gpu.py -x -q --timeout 250 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 || exit 2
echo done
