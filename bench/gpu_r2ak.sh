# A/B of the small trainer step: previous commit (ab_old/, h2a + dW3 wgrad) vs the working tree
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r2ak; mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 120 python -u ab_old/bench/train_bench.py --hidden 256 --batch 65536 --steps 200 --warmup 20 --modes fused >> $O/old.log 2>&1 || exit 1
  timeout -k 10 120 python -u bench/train_bench.py --hidden 256 --batch 65536 --steps 200 --warmup 20 --modes fused >> $O/new.log 2>&1 || exit 2
done
echo done
