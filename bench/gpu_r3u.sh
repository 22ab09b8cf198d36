# round 3: grouped wave tier (several searches per wave) — exactness tests, then route bench A/B of the group width
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r3u; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_astar_gpu.py -m gpu > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 2; }
tail -2 $O/pytest.log
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python -u bench/route_bench.py > $O/rb_$n.log 2>&1 || { tail -20 $O/rb_$n.log; exit 2; }
  echo "$n $(tail -1 $O/rb_$n.log)" | tee -a $O/ab.jsonl
}
run gs16 ROUTEST_ASTAR_WAVE_GROUP=16
run gs32 ROUTEST_ASTAR_WAVE_GROUP=32
run gs64 ROUTEST_ASTAR_WAVE_GROUP=64
