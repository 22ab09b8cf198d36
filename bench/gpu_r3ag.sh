# round 3: 4-wave workgroups per search for the arena reruns and the big tier — exactness tests, 1M-node steps A/B
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r3ag; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_astar_gpu.py -m gpu > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 2; }
tail -1 $O/pytest.log
run() {  # name, args, env...
  local n=$1; local args=$2; shift 2
  env "$@" timeout -k 10 400 python -u bench/astar_scale.py --nodes 1000000 $args > $O/s_$n.log 2>&1 || { tail -20 $O/s_$n.log; exit 3; }
  echo "$n $(tail -1 $O/s_$n.log)" | tee -a $O/ab.jsonl
}
run city_nw4 "--requests 2000 --radius-km 0 --steps 1 --check 4"
run city_nw1 "--requests 2000 --radius-km 0 --steps 1 --check 4" ROUTEST_ASTAR_RETRY_WAVES=1
run local_nw4 "--requests 10000 --radius-km 8"
timeout -k 10 300 python -u bench/route_bench.py > $O/rb.log 2>&1 || { tail -20 $O/rb.log; exit 4; }
tail -1 $O/rb.log
echo done
