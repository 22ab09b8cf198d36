# round 3: lane/wave split by leg length (ROUTEST_ASTAR_LANE_MAX_M) — exactness tests with a split, route bench A/B
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r3x; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_astar_gpu.py -m gpu > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 2; }
tail -2 $O/pytest.log
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python -u bench/route_bench.py > $O/rb_$n.log 2>&1 || { tail -20 $O/rb_$n.log; exit 3; }
  echo "$n $(tail -1 $O/rb_$n.log)" | tee -a $O/ab.jsonl
}
run nosplit
for M in 1000 2000 4000 8000 16000; do run m$M ROUTEST_ASTAR_LANE_MAX_M=$M; done
echo done
