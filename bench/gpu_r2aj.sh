# small trainer: dW3 | db3 inside the forward kernel (two-pass layer 2, no h2a) — tests, bench, stats
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r2aj; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_train_gpu.py tests/test_multirank_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 200 python -u bench/train_bench.py --hidden 256 --batch 65536 --steps 50 --warmup 10 --modes fused,graph > $O/train_h256.log 2>&1 || exit 2
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o train256 --output-format csv -- python3 $ROOT/bench/train_bench.py --hidden 256 --batch 65536 --steps 10 --warmup 3 --modes fused > $O/prof.log 2>&1 || exit 5
echo done
