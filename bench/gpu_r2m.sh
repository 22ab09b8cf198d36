# training defaults (ns=3, KB=64): parity tests incl. wide trainers, DP, train bench
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=gpurun_out/r2m; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_train_gpu.py tests/test_multirank_gpu.py tests/test_mlp_big_gpu.py -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 200 python -u bench/train_bench.py --steps 200 --warmup 20 --modes fused,graph > $O/train_bench.log 2>&1 || exit 2
timeout -k 10 200 python -u bench/train_bench.py --hidden 1024 --batch 16384 --steps 20 --warmup 5 --modes fused > $O/train_bench_h1024.log 2>&1 || exit 3
echo done
