# training step: eager launches vs one captured HIP graph (current kernels), 64k and 1M rows
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r2bc; mkdir -p $O
for i in 1 2; do
for b in 65536 1048576; do
  timeout -k 10 150 python -u bench/train_bench.py --hidden 256 --batch $b --steps 300 --warmup 30 --modes fused,graph >> $O/train.log 2>&1 || exit 1
done
done
echo done
