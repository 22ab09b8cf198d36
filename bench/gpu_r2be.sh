# A* lane-stage pop budget at the config-5 batch (80k legs): 500 (default) vs 250 vs 1 (all wave stage)
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r2be; mkdir -p $O
for r in 1 2; do
for lp in 500 1 250; do
  echo "LANE_POPS=$lp" >> $O/route.log
  ROUTEST_ASTAR_LANE_POPS=$lp timeout -k 10 200 python -u bench/route_bench.py --steps 5 --warmup 1 >> $O/route.log 2>&1 || exit 1
done
done
echo done
