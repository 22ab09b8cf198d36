# round 4: sweep v2 (prefetched records) A/B vs r4c, 16-thread CPU baseline, 1M-node city-wide CCH,
# native history + lifecycle GPU tests, mixed soak, bench.py
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
export TMPDIR=/tmp
O=$ROOT/gpurun_out/r4d; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o cch --output-format csv -- python3 bench/cch_bench.py --reps 3 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
grep cch_legs $O/prof.log
timeout -k 10 120 python -u -m pytest tests/test_cch_gpu.py -x -v --timeout 100 --timeout-method thread > $O/pytest_cch.log 2>&1 || { tail -40 $O/pytest_cch.log; exit 2; }
tail -1 $O/pytest_cch.log
timeout -k 10 300 python3 bench/cch_bench.py --cpu --reps 1 --threads 16 > $O/cch_cpu16.jsonl 2>&1 || { tail -20 $O/cch_cpu16.jsonl; exit 3; }
grep cpu_ $O/cch_cpu16.jsonl
timeout -k 10 400 python -u -m pytest tests/test_native_lifecycle_gpu.py tests/test_frontend_gpu.py -x -v --timeout 240 --timeout-method thread > $O/pytest_native.log 2>&1 || { tail -60 $O/pytest_native.log; exit 4; }
tail -1 $O/pytest_native.log
timeout -k 10 500 python3 bench/astar_scale.py --engine cch --nodes 1000000 --requests 2000 --radius-km 0 --steps 3 > $O/scale_1m.log 2>&1 || { tail -20 $O/scale_1m.log; exit 5; }
tail -1 $O/scale_1m.log
timeout -k 10 300 python3 tools/app_soak.py --stack --clients 128 --seconds 20 > $O/soak.log 2>&1 || { tail -20 $O/soak.log; exit 6; }
tail -1 $O/soak.log | cut -c1-1500
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 7; }
tail -1 $O/bench.log
