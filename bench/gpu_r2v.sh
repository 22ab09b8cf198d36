# global_load_lds weight staging in every per-launch LDS-resident kernel: tests + before/after numbers
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r2v; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_eta_kernel_gpu.py tests/test_gcn_gpu.py tests/test_native_server_gpu.py tests/test_train_gpu.py tests/test_route_scorer.py -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 200 python -u bench/gcn_bench.py --steps 50 --warmup 10 > $O/gcn.log 2>&1 || exit 2
timeout -k 10 200 python -u bench/eta_kernel_sweep.py --batches 4096,65536,1048576,16777216 --variants -1 --iters 20 --rounds 2 > $O/sweep.jsonl 2>&1 || exit 3
timeout -k 10 120 python -u bench/train_bench.py --steps 200 --warmup 20 --modes fused,graph > $O/train.log 2>&1 || exit 4
timeout -k 10 300 python -u bench.py --p50 1 > $O/bench.json 2>$O/bench.err || exit 5
echo done
