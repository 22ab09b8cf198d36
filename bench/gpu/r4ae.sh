# round 4: train_bwd_kernel segment timing with the dgrad (PROF=3) or the dW2 (PROF=4) MFMAs removed (diagnostics)
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
export TMPDIR=/tmp
O=$ROOT/gpurun_out/r4ae; mkdir -p $O
for P in 2 3 4; do
  ROUTEST_TRAIN_BWD_PROF=$P timeout -k 10 150 python3 bench/train_bench.py --hidden 256 --batch 65536 --steps 3 --warmup 2 --modes fused > $O/p$P.log 2>&1 || { tail -20 $O/p$P.log; exit 2; }
  echo "PROF=$P $(grep 'train_bwd prof' $O/p$P.log | tail -1)"
done
