# wide MLP: fused one-launch inference kernel — numerics, A/B vs three-launch path, kernel stats
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=gpurun_out/r2o; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_mlp_big_gpu.py -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
for f in 0 1; do
  ROUTEST_BIG_FUSED=$f timeout -k 10 200 python -u bench/eta_kernel_sweep.py --hidden 512,1024 --batches 1048576,4194304 --variants -1 --iters 5 --rounds 2 > $O/sweep_f$f.jsonl 2>&1 || exit 2
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $ROOT/$O/prof -o sweep --output-format csv -- python3 $ROOT/bench/eta_kernel_sweep.py --hidden 512,1024 --batches 4194304 --variants -1 --iters 5 --rounds 1 > $ROOT/$O/prof.log 2>&1 || exit 4
echo done
