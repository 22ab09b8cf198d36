# Round-end validation on the GPU box: full GPU test suite, smoke(), default bench.py
cd $GRAFT_REPO_ROOT
O=gpurun_out/validate; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 240 python -u -c "import __graft_entry__ as e; e.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 2
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 || exit 3
echo done
