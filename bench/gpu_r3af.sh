# round 3: direct-mapped wave-tier tables (>= N entries, slot = node id) — exactness + route bench A/B
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r3af; mkdir -p $O
ROUTEST_ASTAR_DIRECT=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_astar_gpu.py -m gpu > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 2; }
tail -1 $O/pytest.log
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python -u bench/route_bench.py > $O/rb_$n.log 2>&1 || { tail -20 $O/rb_$n.log; exit 3; }
  echo "$n $(tail -1 $O/rb_$n.log)" | tee -a $O/ab.jsonl
}
run default
run direct_t17 ROUTEST_ASTAR_DIRECT=1 ROUTEST_BULK_WAVE_TBITS=17
run hashed_t17 ROUTEST_BULK_WAVE_TBITS=17
run direct_t17_s32k ROUTEST_ASTAR_DIRECT=1 ROUTEST_BULK_WAVE_TBITS=17 ROUTEST_BULK_WAVE_SLOTS=32768
echo done
