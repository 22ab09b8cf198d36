# round 3: route bench (10k requests, 100k-node graph) A/B of the A* tiering knobs
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r3q; mkdir -p $O
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python -u bench/route_bench.py > $O/rb_$n.log 2>&1 || { tail -20 $O/rb_$n.log; exit 2; }
  echo "$n $(tail -1 $O/rb_$n.log)" | tee -a $O/ab.jsonl
}
run default
run ws65536 ROUTEST_BULK_WAVE_SLOTS=65536
run ws65536_pops1000 ROUTEST_BULK_WAVE_SLOTS=65536 ROUTEST_ASTAR_LANE_POPS=1000
run ws65536_pops250 ROUTEST_BULK_WAVE_SLOTS=65536 ROUTEST_ASTAR_LANE_POPS=250
run ws65536_tb14 ROUTEST_BULK_WAVE_SLOTS=65536 ROUTEST_ASTAR_WAVE_TBITS=14
run wave_only ROUTEST_BULK_WAVE_SLOTS=98304 ROUTEST_ASTAR_WAVE_ONLY_BELOW=1000000
