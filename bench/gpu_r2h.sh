# training: split-K rows per slice A/B (slab traffic vs parallelism)
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=gpurun_out/r2h; mkdir -p $O
for rows in 256 512 1024; do
  ROUTEST_WGRAD_ROWS=$rows timeout -k 10 120 python -u bench/train_bench.py --steps 100 --warmup 20 --modes fused,graph > $O/train_rows$rows.log 2>&1 || exit 1
done
echo done
