# round 6 final, part 1: the whole GPU suite (three parts) with the round-end code
ROOT=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $ROOT
O=$ROOT/gpurun_out/r6o; mkdir -p $O
stop() { rc=$1; [ $rc -eq 124 -o $rc -eq 137 -o $rc -eq 134 -o $rc -eq 139 ] && { echo "GPU step ended rc=$rc: stopping"; exit $rc; }; [ $rc -ne 0 ] && echo "step rc=$rc"; }
A="tests/test_astar_gpu.py tests/test_bench_contract_gpu.py tests/test_cch_gpu.py tests/test_collective_probe_gpu.py tests/test_comm_gpu.py"
B="tests/test_eta_kernel_gpu.py tests/test_frontend_gpu.py tests/test_gcn_gpu.py tests/test_gcn_train_gpu.py tests/test_mlp_big_gpu.py tests/test_multigpu.py tests/test_multirank_gpu.py"
C="tests"; for f in $A $B; do C="$C --ignore=$f"; done
timeout -k 10 420 python -u -m pytest $C -m gpu -v --timeout 240 --timeout-method thread > $O/pytest_C.log 2>&1; stop $?
tail -1 $O/pytest_C.log; grep -E "FAILED|ERROR" $O/pytest_C.log | head
timeout -k 10 360 python -u -m pytest $B -m gpu -v --timeout 240 --timeout-method thread > $O/pytest_B.log 2>&1; stop $?
tail -1 $O/pytest_B.log; grep -E "FAILED|ERROR" $O/pytest_B.log | head
timeout -k 10 400 python -u -m pytest $A -m gpu -v --timeout 240 --timeout-method thread > $O/pytest_A.log 2>&1; stop $?
tail -1 $O/pytest_A.log; grep -E "FAILED|ERROR" $O/pytest_A.log | head
echo done
