set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r1d; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_eta_kernel_gpu.py tests/test_train_gpu.py tests/test_native_server_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || exit 1
timeout -k 10 240 python -u bench/eta_kernel_sweep.py --batches 1048576,4194304,8388608 --variants 3,5,7,8,4,6 > $O/sweep.log 2>&1 || exit 2
timeout -k 10 180 python -u bench.py --p50 0 --io device > $O/bench_dev.log 2>&1 || exit 3
timeout -k 10 180 python -u bench.py > $O/bench_zc.log 2>&1 || exit 4
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/trace_dev -o dev --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --p50 0 --io device > $R/$O/trace_dev.log 2>&1 || exit 5
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/trace_zc -o zc --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --p50 0 > $R/$O/trace_zc.log 2>&1 || exit 6
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY -d $R/$O/pmc -o pmc --output-format csv -- python3 $R/bench/eta_kernel_sweep.py --batches 4194304 --variants 3,5,7 --iters 2 --rounds 1 > $R/$O/pmc.log 2>&1 || exit 7
echo done
