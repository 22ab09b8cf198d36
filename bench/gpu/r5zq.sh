# round 5: per-tile fixed cost of the wide GEMM — time vs K at N = 1024, M = 65536 (both K loops)
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r5zq; mkdir -p $O
for p in 1 0; do
  for K in 512 1024 2048 4096; do
    ROUTEST_GEMM_PIPE=$p timeout -k 10 120 python -u bench/gemm_probe.py --k $K --iters 30 > $O/k${K}_pipe$p.json 2>$O/k${K}_pipe$p.err || { echo "probe K=$K pipe=$p failed rc=$?"; tail -3 $O/k${K}_pipe$p.err; exit 1; }
    echo "pipe=$p $(cat $O/k${K}_pipe$p.json)"
  done
done
