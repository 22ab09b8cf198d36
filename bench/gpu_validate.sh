# Round-end validation on the GPU box: full GPU test suite, smoke(), default bench.py
cd $GRAFT_REPO_ROOT
O=gpurun_out/validate; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 240 python -u -c "import __graft_entry__ as e; e.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 2
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 || exit 3
ROUTEST_BENCH_SHARE_GPU=1 timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 3 --p50 0 > $O/bench_2rank_shared.log 2>&1 || exit 4
echo done
