# wide-MLP training (H = 512, 1024) tests + train bench at H = 1024
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=gpurun_out/r2g; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_train_gpu.py -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 200 python -u bench/train_bench.py --hidden 1024 --batch 16384 --steps 20 --warmup 5 --modes fused,graph > $O/train_bench_h1024.log 2>&1 || exit 2
timeout -k 10 200 python -u bench/train_bench.py --hidden 512 --batch 65536 --steps 20 --warmup 5 --modes fused > $O/train_bench_h512.log 2>&1 || exit 3
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $ROOT/$O/prof -o train1024 --output-format csv -- python3 $ROOT/bench/train_bench.py --hidden 1024 --batch 16384 --steps 10 --warmup 3 --modes fused > $ROOT/$O/prof.log 2>&1 || exit 4
echo done
