# training: dW2 n-block split (fewer slabs) — parity tests, A/B of nsplit, kernel stats
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=gpurun_out/r2k; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_train_gpu.py -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
for ns in 2 3 5 9; do
  ROUTEST_WGRAD_NSPLIT=$ns timeout -k 10 120 python -u bench/train_bench.py --steps 200 --warmup 20 --modes fused > $O/train_ns$ns.log 2>&1 || exit 2
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $ROOT/$O/prof -o train --output-format csv -- python3 $ROOT/bench/train_bench.py --steps 20 --warmup 5 --modes fused > $ROOT/$O/prof.log 2>&1 || exit 4
echo done
