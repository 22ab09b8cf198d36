# training: dW3/dW1 concurrent with dW2 on a side stream — tests, A/B, trace
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=gpurun_out/r2q; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_train_gpu.py tests/test_multirank_gpu.py -k "train or fused or dp" -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
for st in 1 2 1 2; do
  ROUTEST_WGRAD_STREAMS=$st timeout -k 10 120 python -u bench/train_bench.py --steps 200 --warmup 20 --modes fused,graph >> $O/train_st$st.log 2>&1 || exit 2
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $ROOT/$O/prof -o train --output-format csv -- python3 $ROOT/bench/train_bench.py --steps 20 --warmup 5 --modes fused > $ROOT/$O/prof.log 2>&1 || exit 4
echo done
