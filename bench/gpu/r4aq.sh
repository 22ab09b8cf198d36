# round 4: bench.py with the route set-up guarded (agreed on by every rank) — bench contract tests
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
export TMPDIR=/tmp
O=$ROOT/gpurun_out/r4aq; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_bench_contract_gpu.py -x -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 3; }
tail -1 $O/pytest.log
