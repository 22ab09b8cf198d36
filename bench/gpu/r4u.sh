# round 4: register-native dW2 slabs (dwordx4 epilogue) + plain-load slab reduce A/B — train tests, 64k / 1M steps
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
export TMPDIR=/tmp
O=$ROOT/gpurun_out/r4u; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_train_gpu.py -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 2; }
tail -1 $O/pytest.log
for nt in 1 0; do
  ROUTEST_RED_NT=$nt timeout -k 10 150 python3 bench/train_bench.py --hidden 256 --batch 65536 --steps 200 --warmup 20 --modes fused > $O/t64k_nt$nt.log 2>&1 || { tail -20 $O/t64k_nt$nt.log; exit 3; }
  tail -1 $O/t64k_nt$nt.log | cut -c1-300
  ROUTEST_RED_NT=$nt timeout -k 10 150 python3 bench/train_bench.py --hidden 256 --batch 1048576 --steps 40 --warmup 5 --modes fused > $O/t1m_nt$nt.log 2>&1 || { tail -20 $O/t1m_nt$nt.log; exit 4; }
  tail -1 $O/t1m_nt$nt.log | cut -c1-300
done
cd /tmp
timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/prof -o train --output-format csv -- python3 $ROOT/bench/train_bench.py --hidden 256 --batch 65536 --steps 30 --warmup 5 --modes fused > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 5; }
echo prof ok
