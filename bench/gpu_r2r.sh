# wide trainer: dW2 in one wgrad launch (n-blocks in the grid, fewer k-slices) — tests, bench, stats
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=gpurun_out/r2r; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_train_gpu.py -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 200 python -u bench/train_bench.py --hidden 1024 --batch 16384 --steps 50 --warmup 10 --modes fused,graph > $O/train_h1024.log 2>&1 || exit 2
timeout -k 10 200 python -u bench/train_bench.py --hidden 512 --batch 65536 --steps 50 --warmup 10 --modes fused > $O/train_h512.log 2>&1 || exit 3
timeout -k 10 200 python -u bench/train_bench.py --hidden 1024 --batch 65536 --steps 20 --warmup 5 --modes fused > $O/train_h1024_64k.log 2>&1 || exit 4
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $ROOT/$O/prof -o train1024 --output-format csv -- python3 $ROOT/bench/train_bench.py --hidden 1024 --batch 16384 --steps 10 --warmup 3 --modes fused > $ROOT/$O/prof.log 2>&1 || exit 5
echo done
