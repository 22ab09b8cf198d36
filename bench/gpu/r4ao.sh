# round 4: train_bwd fragment prefetch two hidden tiles ahead (PROF 9 = one ahead, the previous form) —
# segment timing, steps, gradient tests
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
export TMPDIR=/tmp
O=$ROOT/gpurun_out/r4ao; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_train_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 6; }
tail -1 $O/pytest.log
for P in 1 9; do
  ROUTEST_TRAIN_BWD_PROF=$P timeout -k 10 150 python3 bench/train_bench.py --hidden 256 --batch 65536 --steps 3 --warmup 2 --modes fused > $O/p$P.log 2>&1 || { tail -20 $O/p$P.log; exit 2; }
  echo "PROF=$P $(grep 'train_bwd prof' $O/p$P.log | tail -1)"
done
timeout -k 10 150 python3 bench/train_bench.py --hidden 256 --batch 65536 --steps 300 --warmup 30 --modes fused > $O/t64k.log 2>&1 || { tail -20 $O/t64k.log; exit 4; }
tail -1 $O/t64k.log | cut -c1-300
timeout -k 10 150 python3 bench/train_bench.py --hidden 256 --batch 1048576 --steps 40 --warmup 5 --modes fused > $O/t1m.log 2>&1 || { tail -20 $O/t1m.log; exit 5; }
tail -1 $O/t1m.log | cut -c1-300
