# round 4: CCH level kernels with the LDS-staged owner search — exactness tests, customization time, kernel table
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
export TMPDIR=/tmp
O=$ROOT/gpurun_out/r4x; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_cch_gpu.py tests/test_frontend_gpu.py -x -v --timeout 200 --timeout-method thread -k "cch or context or graph" > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 2; }
tail -1 $O/pytest.log
timeout -k 10 240 python3 bench/cch_bench.py --reps 2 > $O/cch_bench.jsonl 2>$O/cch_bench.err || { tail -20 $O/cch_bench.err; exit 3; }
grep -E "customiz" $O/cch_bench.jsonl | head -5
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o cch --output-format csv -- python3 $ROOT/bench/cch_bench.py --reps 2 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 4; }
echo prof ok
