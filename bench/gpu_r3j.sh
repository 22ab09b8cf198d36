# round 3: training step v3 — single-pass forward (relu(z2) kept packed, dW3 by MFMA transposes) +
# one fused backward kernel (dgrad + relu'(z1) + dW2 + dW1, dz2 image read row-wise and transposed)
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/${TAG:-r3j}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_train_gpu.py -x -q --timeout 240 --timeout-method thread > $O/pytest_train.log 2>&1 || { tail -60 $O/pytest_train.log; exit 1; }
tail -2 $O/pytest_train.log
for B in 65536 262144 1048576; do
  timeout -k 10 120 python -u bench/train_bench.py --hidden 256 --batch $B --steps 30 --warmup 5 --modes fused > $O/tb_$B.log 2>&1 || { tail -20 $O/tb_$B.log; exit 4; }
  echo "B=$B $(tail -1 $O/tb_$B.log)" | tee -a $O/train.jsonl
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/train1m -o train --output-format csv -- python3 $ROOT/bench/train_bench.py --hidden 256 --batch 1048576 --steps 10 --warmup 3 --modes fused > $O/train1m.log 2>&1 || exit 31
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/train64k -o train --output-format csv -- python3 $ROOT/bench/train_bench.py --hidden 256 --batch 65536 --steps 20 --warmup 3 --modes fused > $O/train64k.log 2>&1 || exit 32
echo done
