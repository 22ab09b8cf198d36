# dual wgrad launch (dW2|db2 + dW1 in one grid): training numerics, A/B step time, kernel stats
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r2as; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_train_gpu.py tests/test_multirank_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
for i in 1 2 3; do
  ROUTEST_WGRAD_DUAL=0 timeout -k 10 120 python -u bench/train_bench.py --hidden 256 --batch 65536 --steps 300 --warmup 30 --modes fused >> $O/dual0.log 2>&1 || exit 2
  ROUTEST_WGRAD_DUAL=1 timeout -k 10 120 python -u bench/train_bench.py --hidden 256 --batch 65536 --steps 300 --warmup 30 --modes fused >> $O/dual1.log 2>&1 || exit 3
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o train --output-format csv -- python3 $ROOT/bench/train_bench.py --hidden 256 --batch 65536 --steps 50 --warmup 5 --modes fused > $O/prof.log 2>&1 || exit 4
echo done
