# K3 forward with fused relu'(z1): training tests + bench + kernel stats
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=gpurun_out/r2i; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_train_gpu.py tests/test_multirank_gpu.py -k "train or fused or adam or pack or wgrad or dp or wide" -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 200 python -u bench/train_bench.py --steps 100 --warmup 20 --modes fused,graph > $O/train_bench.log 2>&1 || exit 3
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $ROOT/$O/prof -o train --output-format csv -- python3 $ROOT/bench/train_bench.py --steps 20 --warmup 5 --modes fused > $ROOT/$O/prof.log 2>&1 || exit 4
echo done
