# wide MLP: 256x256 glds GEMM — numerics tests, A/B vs the 128x128 kernel, H=1024 training, kernel stats
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=gpurun_out/r2n; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_mlp_big_gpu.py tests/test_train_gpu.py -k "big or wide or 512 or 1024" -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
for t in 128 256; do
  ROUTEST_GEMM_TILE=$t timeout -k 10 200 python -u bench/eta_kernel_sweep.py --hidden 512,1024 --batches 1048576,4194304 --variants -1 --iters 5 --rounds 2 > $O/sweep_t$t.jsonl 2>&1 || exit 2
  ROUTEST_GEMM_TILE=$t timeout -k 10 200 python -u bench/train_bench.py --hidden 1024 --batch 16384 --steps 20 --warmup 5 --modes fused > $O/train1024_t$t.log 2>&1 || exit 3
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $ROOT/$O/prof -o sweep --output-format csv -- python3 $ROOT/bench/eta_kernel_sweep.py --hidden 1024 --batches 4194304 --variants -1 --iters 5 --rounds 1 > $ROOT/$O/prof.log 2>&1 || exit 4
echo done
