# training: dz2 kept in registers, rebuilt by the dW2 wgrad from h2a (33.5 MB fewer writes) — tests, bench, PMC
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r2ac; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_train_gpu.py tests/test_multirank_gpu.py -k "train or fused or dp or wgrad" -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 120 python -u bench/train_bench.py --steps 200 --warmup 20 --modes fused,graph > $O/train.log 2>&1 || exit 2
timeout -k 10 120 python -u bench/train_bench.py --steps 200 --warmup 20 --modes fused,graph >> $O/train.log 2>&1 || exit 2
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES -d $O/pmc -o g --output-format csv -- python3 $ROOT/bench/train_bench.py --steps 5 --warmup 2 --modes fused > $O/pmc.log 2>&1 || exit 3
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o train --output-format csv -- python3 $ROOT/bench/train_bench.py --steps 20 --warmup 5 --modes fused > $O/prof.log 2>&1 || exit 4
echo done
