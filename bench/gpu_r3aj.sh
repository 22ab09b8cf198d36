# round 3: route step with 98304 wave-tier slots (one launch for every escalated leg) vs 65536
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r3aj; mkdir -p $O
rb() {
  local n=$1; shift
  env "$@" timeout -k 10 300 python -u bench/route_bench.py > $O/rb_$n.log 2>&1 || { tail -20 $O/rb_$n.log; exit 4; }
  echo "$n $(tail -1 $O/rb_$n.log)" | tee -a $O/ab.jsonl
}
rb slots65536
rb slots98304 ROUTEST_BULK_WAVE_SLOTS=98304
timeout -k 10 300 python -u bench/astar_ab.py > $O/ab_tiers.log 2>&1 || { tail -20 $O/ab_tiers.log; exit 5; }
tail -3 $O/ab_tiers.log
echo done
