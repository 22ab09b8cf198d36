# round 4: CCH kernel profile + native route/lifecycle GPU tests + bench.py
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
export TMPDIR=/tmp
O=$ROOT/gpurun_out/r4c; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o cch --output-format csv -- python3 bench/cch_bench.py --reps 2 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
ls -R $O/prof > $O/prof_files.txt
timeout -k 10 300 python3 bench/cch_bench.py --cpu --reps 2 > $O/cch_cpu.jsonl 2>&1 || { tail -20 $O/cch_cpu.jsonl; exit 4; }
tail -2 $O/cch_cpu.jsonl
timeout -k 10 600 python -u -m pytest tests/test_native_lifecycle_gpu.py tests/test_frontend_gpu.py -x -v --timeout 240 --timeout-method thread > $O/pytest_native.log 2>&1 || { tail -80 $O/pytest_native.log; exit 2; }
tail -3 $O/pytest_native.log
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 3; }
tail -1 $O/bench.log
