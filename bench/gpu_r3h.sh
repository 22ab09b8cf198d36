# round 3: training backward redesign v2 (MFMA transpose, prefetching buffer-load wgrad) — numerics, bench, stats
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r3h2; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_train_gpu.py -x -q --timeout 240 --timeout-method thread > $O/pytest_train.log 2>&1 || { tail -60 $O/pytest_train.log; exit 1; }
tail -2 $O/pytest_train.log
for B in 65536 1048576; do
  for T in 4 8 16; do
    ROUTEST_TRAIN_WGRAD_TILES=$T timeout -k 10 120 python -u bench/train_bench.py --hidden 256 --batch $B --steps 30 --warmup 5 --modes fused > $O/tb_${B}_$T.log 2>&1 || { tail -20 $O/tb_${B}_$T.log; exit 2; }
    echo "B=$B tiles=$T $(tail -1 $O/tb_${B}_$T.log)" | tee -a $O/train.jsonl
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/train1m -o train --output-format csv -- python3 $ROOT/bench/train_bench.py --hidden 256 --batch 1048576 --steps 10 --warmup 3 --modes fused > $O/train1m.log 2>&1 || exit 31
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/train64k -o train --output-format csv -- python3 $ROOT/bench/train_bench.py --hidden 256 --batch 65536 --steps 20 --warmup 3 --modes fused > $O/train64k.log 2>&1 || exit 32
cd $ROOT
timeout -k 10 600 python -u bench/astar_ab.py > $O/astar_ab.log 2>&1 || { tail -20 $O/astar_ab.log; exit 5; }
cat $O/astar_ab.log | grep config
echo done
