# 6-byte vs 8-byte wire records: kernel tests + headline A/B + default bench (run on the GPU box)
cd $GRAFT_REPO_ROOT
O=gpurun_out/rec6; mkdir -p $O; rm -f $O/*.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_eta_kernel_gpu.py tests/test_bench_contract_gpu.py > $O/tests.log 2>&1 || exit 1
for r in 6 8; do
  timeout -k 10 200 python -u bench.py --rec $r --p50 0 >> $O/bench_$r.log 2>&1 || exit 2
done
timeout -k 10 300 python -u bench.py > $O/bench_default.log 2>&1 || exit 3
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $GRAFT_REPO_ROOT/$O/trace -o rec6 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --p50 0 > $GRAFT_REPO_ROOT/$O/trace.log 2>&1 || exit 4
echo done
