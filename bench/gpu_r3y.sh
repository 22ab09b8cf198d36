# round 3: lane-split default (8 median edges) — A* + route-service tests, route bench threshold sweep
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r3y; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_astar_gpu.py tests/test_frontend_gpu.py tests/test_route_batcher_gpu.py -m gpu > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 2; }
tail -2 $O/pytest.log
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python -u bench/route_bench.py > $O/rb_$n.log 2>&1 || { tail -20 $O/rb_$n.log; exit 3; }
  echo "$n $(tail -1 $O/rb_$n.log)" | tee -a $O/ab.jsonl
}
run default
for M in 1 250 500 700; do run m$M ROUTEST_ASTAR_LANE_MAX_M=$M; done
run default2
echo done
