# Headline with the auto-selected 16x16-MFMA kernel: kernel tests, default bench.py x2, kernel trace
cd $GRAFT_REPO_ROOT
O=gpurun_out/h16; mkdir -p $O; rm -f $O/*.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_eta_kernel_gpu.py tests/test_bench_contract_gpu.py tests/test_native_server_gpu.py > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > $O/bench_default.log 2>&1 || exit 2
timeout -k 10 200 python -u bench.py --p50 0 > $O/bench_nop50.log 2>&1 || exit 3
timeout -k 10 200 python -u bench.py --p50 0 --variant 3 > $O/bench_v3.log 2>&1 || exit 4
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $GRAFT_REPO_ROOT/$O/trace -o h16 --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --p50 0 > $GRAFT_REPO_ROOT/$O/trace.log 2>&1 || exit 5
echo done
