# training forward: dW3 partial on the transposed layer-2 tile (in-lane row sums) — numerics + A/B vs ab_old (HEAD)
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r2aw; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_train_gpu.py tests/test_multirank_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
for i in 1 2 3; do
  timeout -k 10 120 python -u ab_old/bench/train_bench.py --hidden 256 --batch 65536 --steps 300 --warmup 30 --modes fused >> $O/old.log 2>&1 || exit 2
  timeout -k 10 120 python -u bench/train_bench.py --hidden 256 --batch 65536 --steps 300 --warmup 30 --modes fused >> $O/new.log 2>&1 || exit 3
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o train --output-format csv -- python3 $ROOT/bench/train_bench.py --hidden 256 --batch 65536 --steps 50 --warmup 5 --modes fused > $O/prof.log 2>&1 || exit 4
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS -d $O/pmc -o train --output-format csv -- python3 $ROOT/bench/train_bench.py --hidden 256 --batch 65536 --steps 5 --warmup 2 --modes fused > $O/pmc.log 2>&1 || exit 5
echo done
