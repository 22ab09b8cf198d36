# A* wave-stage f-band width (ROUTEST_ASTAR_DELTA, seconds) at the config-5 batch
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r2bf; mkdir -p $O
for r in 1 2; do
for d in 10 5 20 40; do
  echo "DELTA=$d" >> $O/route.log
  ROUTEST_ASTAR_DELTA=$d timeout -k 10 200 python -u bench/route_bench.py --steps 5 --warmup 1 >> $O/route.log 2>&1 || exit 1
done
done
echo done
