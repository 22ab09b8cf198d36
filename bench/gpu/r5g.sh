# round 5: watchdog rehearsal (armed isolated streams) + the whole GPU suite in two parts
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r5g; mkdir -p $O
stop() { rc=$1; [ $rc -eq 124 -o $rc -eq 137 -o $rc -eq 134 -o $rc -eq 139 ] && { echo "GPU step ended rc=$rc: stopping"; exit $rc; }; [ $rc -ne 0 ] && echo "step rc=$rc"; }
timeout -k 10 170 python -u -m pytest -x -v -s --timeout 160 --timeout-method thread tests/test_native_lifecycle_gpu.py -k hung > $O/watchdog.log 2>&1; stop $?
timeout -k 10 500 python -u -m pytest -v -m gpu --timeout 240 --timeout-method thread tests/test_eta_kernel_gpu.py tests/test_train_gpu.py tests/test_mlp_big_gpu.py tests/test_forest.py tests/test_gcn_gpu.py tests/test_gcn_train_gpu.py tests/test_gcn_observed.py tests/test_comm_gpu.py tests/test_collective_probe_gpu.py tests/test_multirank_gpu.py tests/test_elastic.py tests/test_route_kernels_gpu.py tests/test_astar_gpu.py > $O/suite_a.log 2>&1; stop $?
echo done
