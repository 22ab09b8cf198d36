# round 3: 100k route step with the lane split, wave-tier ordering on / off
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r3ab; mkdir -p $O
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python -u bench/route_bench.py > $O/rb_$n.log 2>&1 || { tail -20 $O/rb_$n.log; exit 3; }
  echo "$n $(tail -1 $O/rb_$n.log)" | tee -a $O/ab.jsonl
}
run split_nolpt ROUTEST_ASTAR_LPT=0
run split_lpt
run split_nolpt2 ROUTEST_ASTAR_LPT=0
echo done
