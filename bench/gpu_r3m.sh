# round 3: k-slice sizing sweep of train_bwd_kernel (ROUTEST_TRAIN_WGRAD_TILES = min tiles per slice)
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r3m; mkdir -p $O
for B in 65536 1048576; do
  for T in 4 8 12 16; do
    ROUTEST_TRAIN_WGRAD_TILES=$T timeout -k 10 120 python -u bench/train_bench.py --hidden 256 --batch $B --steps 30 --warmup 5 --modes fused > $O/tb_${B}_$T.log 2>&1 || { tail -20 $O/tb_${B}_$T.log; exit 2; }
    echo "B=$B tiles=$T $(tail -1 $O/tb_${B}_$T.log)" | tee -a $O/train.jsonl
  done
done
for H in 1024 512; do
  timeout -k 10 120 python -u bench/train_bench.py --hidden $H --batch 65536 --steps 20 --warmup 3 --modes fused > $O/tbw_$H.log 2>&1 || { tail -20 $O/tbw_$H.log; exit 3; }
  echo "H=$H $(tail -1 $O/tbw_$H.log)" | tee -a $O/train.jsonl
done
