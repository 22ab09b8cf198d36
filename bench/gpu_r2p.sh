# fused wide kernel: 3 W2 stages (counted vmcnt + raw barrier) vs 2 — numerics + A/B
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=gpurun_out/r2p; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_mlp_big_gpu.py -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
for ns in 2 3; do
  ROUTEST_BIG_STAGES=$ns timeout -k 10 200 python -u bench/eta_kernel_sweep.py --hidden 512,1024 --batches 1048576,4194304 --variants -1 --iters 5 --rounds 3 > $O/sweep_ns$ns.jsonl 2>&1 || exit 2
done
echo done
