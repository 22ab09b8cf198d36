# round 4: GPU CCH correctness + first timings
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
export TMPDIR=/tmp
O=$ROOT/gpurun_out/r4b; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_cch_gpu.py -x -v --timeout 240 --timeout-method thread > $O/pytest_cch.log 2>&1 || { tail -60 $O/pytest_cch.log; exit 1; }
tail -5 $O/pytest_cch.log
timeout -k 10 400 python -u bench/cch_bench.py --astar --cpu > $O/cch_bench.jsonl 2>&1 || { tail -30 $O/cch_bench.jsonl; exit 2; }
cat $O/cch_bench.jsonl
