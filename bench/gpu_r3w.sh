# round 3: longest-first wave-tier ordering — exactness tests, route bench A/B (LPT on/off), 1M-node step,
# plus the wide-trainer (H = 1024) kernel stats as CSV
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
export TMPDIR=/tmp
O=$ROOT/gpurun_out/r3w; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_astar_gpu.py -m gpu > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 2; }
tail -2 $O/pytest.log
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python -u bench/route_bench.py > $O/rb_$n.log 2>&1 || { tail -20 $O/rb_$n.log; exit 3; }
  echo "$n $(tail -1 $O/rb_$n.log)" | tee -a $O/ab.jsonl
}
run lpt
run query_order ROUTEST_ASTAR_LPT=0
run lpt2
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o h1024 --output-format csv -- python3 bench/train_bench.py --hidden 1024 --batch 65536 --steps 10 --warmup 2 --modes fused > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 4; }
echo done
