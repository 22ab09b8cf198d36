# wide trainer: fused dy+dz2+step kernel, tiled W2 AdamW — tests, benches, stats
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r2ai; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_train_gpu.py tests/test_mlp_big_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 200 python -u bench/train_bench.py --hidden 1024 --batch 16384 --steps 50 --warmup 10 --modes fused,graph > $O/train_h1024.log 2>&1 || exit 2
timeout -k 10 200 python -u bench/train_bench.py --hidden 512 --batch 65536 --steps 50 --warmup 10 --modes fused > $O/train_h512.log 2>&1 || exit 3
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o train1024 --output-format csv -- python3 $ROOT/bench/train_bench.py --hidden 1024 --batch 16384 --steps 10 --warmup 3 --modes fused > $O/prof.log 2>&1 || exit 5
echo done
