# dual wgrad launch: n-blocks per k-slice for dW2 (ROUTEST_WGRAD_NSPLIT) re-swept
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r2bk; mkdir -p $O
for r in 1 2; do
for ns in 3 2 5 9; do
  echo "NSPLIT=$ns" >> $O/train.log
  ROUTEST_WGRAD_NSPLIT=$ns timeout -k 10 120 python -u bench/train_bench.py --hidden 256 --batch 65536 --steps 300 --warmup 30 --modes fused >> $O/train.log 2>&1 || exit 1
done
done
echo done
