# registered host buffers test + multi-rank rehearsal with the round-2 kernels
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r2w; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_eta_kernel_gpu.py -k "registered or zero_copy or mixed" tests/test_multirank_gpu.py tests/test_collective_probe_gpu.py tests/test_bench_contract_gpu.py -x -v --timeout 250 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
export ROUTEST_BENCH_SHARE_GPU=1
timeout -k 10 200 python -u bench/train_bench.py --gpus 2 --steps 20 --warmup 3 --modes fused --comm oneshot > $O/train_2rank_shared.log 2>&1 || exit 2
timeout -k 10 200 python -u bench.py --gpus 2 --steps 5 --warmup 2 --batch 1048576 --p50 0 > $O/bench_2rank_shared.log 2>&1 || exit 3
echo done
