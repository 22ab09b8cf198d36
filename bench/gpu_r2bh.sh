# end-of-session validation: full GPU suite, smoke, default bench, 2-rank shared bench, app soak
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=gpurun_out/r2bh; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=15 > $O/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 240 python -u -c "import __graft_entry__ as e; e.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 2
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 || exit 3
ROUTEST_BENCH_SHARE_GPU=1 timeout -k 10 300 python -u bench.py --gpus 2 --steps 10 --warmup 3 --p50 0 > $O/bench_2rank_shared.log 2>&1 || exit 4
timeout -k 10 200 python -u tools/app_soak.py --seconds 30 --clients 64 > $O/soak.log 2>&1 || exit 5
echo done
