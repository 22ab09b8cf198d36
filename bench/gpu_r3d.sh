# round 3: lane-stage budget sweep for the native graph route path (ROUTEST_ASTAR_LANE_POPS)
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r3d; mkdir -p $O
for lp in 1 100 2000; do
  ROUTEST_ASTAR_LANE_POPS=$lp timeout -k 10 300 python -u bench/route_http_bench.py --provider graph --modes native --seconds 6 > $O/route_graph_lp$lp.log 2>&1 || { tail -30 $O/route_graph_lp$lp.log; exit 3; }
  echo "lane_pops=$lp"; tail -1 $O/route_graph_lp$lp.log | python -c "import json,sys; d=json.load(sys.stdin)['native']; print(round(d['req_per_s']), d['p50_ms'], d['stage_ms_per_flush'])"
done
echo done
