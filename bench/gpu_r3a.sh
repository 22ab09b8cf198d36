# round 3 first pass: full GPU suite (8-byte wire records, new checkpoint format) + default bench line
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r3a; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { tail -50 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 2; }
tail -c 3000 $O/bench.log
echo done
