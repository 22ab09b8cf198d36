# round 3: route bench (10k requests, 100k-node graph) A/B of the wave-tier band width and table size
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r3s; mkdir -p $O
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python -u bench/route_bench.py > $O/rb_$n.log 2>&1 || { tail -20 $O/rb_$n.log; exit 2; }
  echo "$n $(tail -1 $O/rb_$n.log)" | tee -a $O/ab.jsonl
}
run default
run delta5 ROUTEST_ASTAR_DELTA=5
run delta20 ROUTEST_ASTAR_DELTA=20
run delta40 ROUTEST_ASTAR_DELTA=40
run tb15 ROUTEST_BULK_WAVE_TBITS=15
run pops750 ROUTEST_ASTAR_LANE_POPS=750
