# round 4: the whole GPU test suite (what the driver runs at round end) + smoke
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
export TMPDIR=/tmp
O=$ROOT/gpurun_out/r4t; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { tail -80 $O/pytest.log; exit 2; }
tail -1 $O/pytest.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 3; }
tail -1 $O/smoke.log
