# round 3: train_bwd_kernel per-segment s_memtime profile (ROUTEST_TRAIN_BWD_PROF=1; =2: the same
# without the hidden-tile loop's LDS reads, timing only) at 1M rows
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r3o; mkdir -p $O
for P in 1 2 3 4; do
  ROUTEST_TRAIN_BWD_PROF=$P timeout -k 10 120 python -u bench/train_bench.py --hidden 256 --batch 1048576 --steps 2 --warmup 1 --modes fused > $O/prof_$P.log 2>&1 || { tail -20 $O/prof_$P.log; exit 2; }
  echo "mode $P: $(grep 'train_bwd prof' $O/prof_$P.log | tail -1)"
done
