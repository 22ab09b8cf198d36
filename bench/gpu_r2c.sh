# multi-rank paths on one GPU: one-shot all-gather/broadcast, GCN partition, DP trainer, 2-runner batcher;
# benches launching their own ranks (shared-GPU rehearsal)
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=gpurun_out/r2c; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_multirank_gpu.py tests/test_comm_gpu.py tests/test_gcn_gpu.py tests/test_bench_contract_gpu.py -x -v --timeout 280 -k "batcher or gcn or bench"  --timeout-method thread > $O/pytest.log 2>&1 || exit 1
export ROUTEST_BENCH_SHARE_GPU=1
timeout -k 10 200 python -u bench/gcn_bench.py --gpus 2 --steps 20 --warmup 3 > $O/gcn_2rank_shared.log 2>&1 || exit 2
timeout -k 10 200 python -u bench/train_bench.py --gpus 2 --steps 20 --warmup 3 --modes fused --comm oneshot > $O/train_2rank_shared.log 2>&1 || exit 3
timeout -k 10 200 python -u bench.py --gpus 4 --steps 5 --warmup 2 --batch 1048576 --p50 0 > $O/bench_4rank_shared.log 2>&1 || exit 4
echo done
