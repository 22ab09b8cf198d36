# K3 fused dgrad re-verification + wide MLP (H = 512, 1024) tests and sweep
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=gpurun_out/r2f; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_train_gpu.py tests/test_multirank_gpu.py tests/test_mlp_big_gpu.py tests/test_eta_kernel_gpu.py -k "not experimental" -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 200 python -u bench/train_bench.py --steps 50 --warmup 10 --modes fused,graph > $O/train_bench.log 2>&1 || exit 3
timeout -k 10 300 python -u bench/eta_kernel_sweep.py --hidden 512,1024 --batches 1048576,4194304 --variants -1 --iters 5 --rounds 2 > $O/sweep_big.jsonl 2>&1 || exit 4
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $ROOT/$O/prof -o train --output-format csv -- python3 $ROOT/bench/train_bench.py --steps 20 --warmup 5 --modes fused > $ROOT/$O/prof.log 2>&1 || exit 5
echo done
