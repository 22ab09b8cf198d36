# round 3: wide trainer with dW3 folded into big_dz2y — gradients vs autograd, H = 512 / 1024 step times, kernel stats
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
export TMPDIR=/tmp
O=$ROOT/gpurun_out/r3ad; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_train_gpu.py -m gpu > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 2; }
tail -2 $O/pytest.log
for H in 1024 512; do
  for B in 16384 65536 262144; do
    timeout -k 10 180 python -u bench/train_bench.py --hidden $H --batch $B --steps 20 --warmup 3 --modes fused > $O/tb_${H}_$B.log 2>&1 || { tail -20 $O/tb_${H}_$B.log; exit 3; }
    echo "H=$H B=$B $(tail -1 $O/tb_${H}_$B.log)" | tee -a $O/train.jsonl
  done
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o h1024 --output-format csv -- python3 bench/train_bench.py --hidden 1024 --batch 65536 --steps 10 --warmup 2 --modes fused > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 4; }
echo done
