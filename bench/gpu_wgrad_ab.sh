set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/wg; mkdir -p $O
for kb in 32 64 128; do
  ROUTEST_WGRAD_KB=$kb timeout -k 10 200 python -u -m pytest tests/test_train_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "wgrad or gradients" > $O/t_$kb.log 2>&1 || exit 1
  for rows in 256 512; do
    ROUTEST_WGRAD_KB=$kb ROUTEST_WGRAD_ROWS=$rows timeout -k 10 120 python -u bench/train_bench.py --modes fused > $O/b_${kb}_$rows.log 2>&1 || exit 2
  done
done
echo done
