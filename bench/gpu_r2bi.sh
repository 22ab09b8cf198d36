# headline IO A/B on one box: hybrid (DMA in, zero-copy minutes out) vs host (DMA both ways), 6-byte records
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r2bi; mkdir -p $O
for i in 1 2 3; do
for io in hybrid host; do
  timeout -k 10 200 python -u bench.py --io $io --steps 100 --warmup 10 --p50 0 --rec16-steps 0 --train-steps 0 --gcn-steps 0 --route-steps 0 >> $O/$io.log 2>&1 || exit 1
done
done
echo done
