# full GPU suite + smoke + default bench at HEAD (batcher queue fix, elastic tests, transposed dW3)
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=gpurun_out/r2ba; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=15 > $O/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 240 python -u -c "import __graft_entry__ as e; e.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 2
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 || exit 3
echo done
