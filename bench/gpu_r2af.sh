# headline kernel: layer 3 on MFMA (variant 23) — tests, A/B vs 17/20 (6- and 16-byte records), bench
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r2af; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_eta_kernel_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 200 python -u bench/eta_kernel_sweep.py --batches 16777216 --variants 17,20,23 --iters 10 --rounds 3 > $O/sweep16.jsonl 2>&1 || exit 2
timeout -k 10 200 python -u bench/eta_kernel_sweep.py --batches 16777216 --variants 17,20,23 --iters 10 --rounds 3 --rec 6 > $O/sweep6.jsonl 2>&1 || exit 3
timeout -k 10 300 python -u bench.py --variant 23 --p50 0 > $O/bench23.json 2> $O/bench23.err || exit 4
timeout -k 10 300 python -u bench.py --variant 20 --p50 0 > $O/bench20.json 2> $O/bench20.err || exit 5
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES -d $O/pmc -o g --output-format csv -- python3 $ROOT/bench/eta_kernel_sweep.py --batches 8388608 --variants 20,23 --iters 3 --rounds 1 > $O/pmc.log 2>&1 || exit 6
echo done
