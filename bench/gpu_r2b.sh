# fwd16 epilogue A/B: 17 (packed f32 epilogue) vs 20 (scalar FMA) vs 21 (scalar, pipelined) vs 22 (21, 2 halves)
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=gpurun_out/r2b; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_eta_kernel_gpu.py -x -q --timeout 150 --timeout-method thread -k "matches_fp32 or rec6" > $O/pytest.log 2>&1 || exit 1
for rec in 6 16; do
timeout -k 10 200 python -u bench/eta_kernel_sweep.py --batches 16777216 --variants 17,20,21,22,3 --iters 10 --rounds 3 --rec $rec > $O/sweep_rec$rec.jsonl 2>&1 || exit 2
done
for v in 17 20 21; do
timeout -k 10 200 python -u bench.py --variant $v --p50 0 --rec16-steps 0 > $O/bench_v$v.log 2>&1 || exit 3
done
echo done
