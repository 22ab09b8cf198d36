# one-shot collectives with the fused stage+signal kernel: comm + multi-rank suites, 2-rank shared bench
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=gpurun_out/r2ao; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_comm_gpu.py tests/test_multirank_gpu.py tests/test_collective_probe_gpu.py -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
ROUTEST_BENCH_SHARE_GPU=1 timeout -k 10 300 python -u bench.py --gpus 2 --steps 10 --warmup 3 --p50 0 > $O/bench_2rank_shared.log 2>&1 || exit 2
echo done
