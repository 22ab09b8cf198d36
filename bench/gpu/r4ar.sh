# round 4: final bench.py line (no flags) on the round-end code + bench contract tests
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
export TMPDIR=/tmp
O=$ROOT/gpurun_out/r4ar; mkdir -p $O
timeout -k 10 900 python -u bench.py > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 2; }
tail -1 $O/bench.log | cut -c1-300
timeout -k 10 600 python -u -m pytest tests/test_bench_contract_gpu.py -x -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 3; }
tail -1 $O/pytest.log
