# bench.py with the config-5 route probe: contract tests, refactored route_bench, full default bench (timed)
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=gpurun_out/r2an; mkdir -p $O
#timeout -k 10 300 python -u -m pytest tests/test_bench_contract_gpu.py -k route -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
#timeout -k 10 200 python -u bench/route_bench.py --steps 5 --warmup 1 > $O/route.log 2>&1 || exit 2
s0=$SECONDS; timeout -k 10 400 python -u bench.py > $O/bench.log 2> $O/bench.err || exit 3; echo "bench wall $((SECONDS-s0)) s" > $O/bench_wall.txt

for b in 65536 262144 1048576; do
timeout -k 10 200 python -u bench/train_bench.py --hidden 256 --batch $b --steps 100 --warmup 10 --modes fused >> $O/train_batch.log 2>&1 || exit 4
done
echo done
