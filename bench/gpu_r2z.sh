# fused wide kernel: s_setprio around MFMA bursts A/B
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r2z; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_mlp_big_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
for p in 0 1 0 1; do
  ROUTEST_BIG_PRIO=$p timeout -k 10 200 python -u bench/eta_kernel_sweep.py --hidden 512,1024 --batches 4194304 --variants -1 --iters 5 --rounds 3 >> $O/sweep_p$p.jsonl 2>&1 || exit 2
done
echo done
