# round 5: latency watchdog (gpu_hang@1 on a 2-slot shared-GPU rehearsal), multi-GPU readiness
# rehearsal (tests/test_multigpu.py + bench.py --gpus 2, both with every rank on GPU 0)
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r5b; mkdir -p $O
stop() { rc=$1; [ $rc -eq 124 -o $rc -eq 137 -o $rc -eq 134 -o $rc -eq 139 ] && { echo "GPU step ended rc=$rc: stopping"; exit $rc; }; }
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 250 --timeout-method thread tests/test_native_lifecycle_gpu.py -k hung > $O/watchdog.log 2>&1; stop $?
timeout -k 10 500 env ROUTEST_TEST_SHARE_GPU=1 python -u -m pytest -x -v --timeout 450 --timeout-method thread tests/test_multigpu.py > $O/multigpu_share.log 2>&1; stop $?
timeout -k 10 240 env ROUTEST_BENCH_SHARE_GPU=1 python bench.py --gpus 2 --steps 10 --warmup 3 --p50 0 > $O/bench_share2.log 2>&1; stop $?
echo done
