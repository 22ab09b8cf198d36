# round 3: 1M-node local step — which of the wave-tier ordering / lane split caused the 1452 -> 1630 ms change
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r3aa; mkdir -p $O
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python -u bench/astar_scale.py --nodes 1000000 --requests 10000 --radius-km 8 > $O/s_$n.log 2>&1 || { tail -20 $O/s_$n.log; exit 3; }
  echo "$n $(tail -1 $O/s_$n.log)" | tee -a $O/ab.jsonl
}
run lpt_nosplit ROUTEST_ASTAR_LANE_MAX_M=0
run nolpt_nosplit ROUTEST_ASTAR_LANE_MAX_M=0 ROUTEST_ASTAR_LPT=0
run nolpt_split ROUTEST_ASTAR_LPT=0
echo done
