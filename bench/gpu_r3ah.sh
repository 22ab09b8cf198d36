# round 3: waves per search — main wave tier (ROUTEST_ASTAR_WAVE_WAVES) and reruns (ROUTEST_ASTAR_RETRY_WAVES)
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r3ah; mkdir -p $O
ROUTEST_ASTAR_WAVE_WAVES=2 ROUTEST_ASTAR_RETRY_WAVES=8 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_astar_gpu.py -m gpu > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 2; }
tail -1 $O/pytest.log
run() {  # name, args, env...
  local n=$1; local args=$2; shift 2
  env "$@" timeout -k 10 400 python -u bench/astar_scale.py --nodes 1000000 $args > $O/s_$n.log 2>&1 || { tail -20 $O/s_$n.log; exit 3; }
  echo "$n $(tail -1 $O/s_$n.log)" | tee -a $O/ab.jsonl
}
run city_r8 "--requests 2000 --radius-km 0 --steps 1 --check 4" ROUTEST_ASTAR_RETRY_WAVES=8
run local_w2 "--requests 10000 --radius-km 8" ROUTEST_ASTAR_WAVE_WAVES=2
run local_w4 "--requests 10000 --radius-km 8" ROUTEST_ASTAR_WAVE_WAVES=4
rb() {
  local n=$1; shift
  env "$@" timeout -k 10 300 python -u bench/route_bench.py > $O/rb_$n.log 2>&1 || { tail -20 $O/rb_$n.log; exit 4; }
  echo "$n $(tail -1 $O/rb_$n.log)" | tee -a $O/ab.jsonl
}
rb rb_w1
rb rb_w2 ROUTEST_ASTAR_WAVE_WAVES=2
echo done
