# round 4 final check (after the route_core put_coord fix): the whole GPU suite in three parts and smoke
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
export TMPDIR=/tmp
O=$ROOT/gpurun_out/r4au; mkdir -p $O
A="tests/test_astar_gpu.py tests/test_bench_contract_gpu.py tests/test_cch_gpu.py tests/test_collective_probe_gpu.py tests/test_comm_gpu.py"
B="tests/test_eta_kernel_gpu.py tests/test_frontend_gpu.py tests/test_gcn_gpu.py tests/test_gcn_train_gpu.py tests/test_mlp_big_gpu.py tests/test_multigpu.py tests/test_multirank_gpu.py"
C="tests"; for f in $A $B; do C="$C --ignore=$f"; done
timeout -k 10 300 python -u -m pytest $C -m gpu -v --timeout 240 --timeout-method thread > $O/pytest_C.log 2>&1 || { tail -60 $O/pytest_C.log; exit 5; }
tail -1 $O/pytest_C.log
timeout -k 10 300 python -u -m pytest $B -m gpu -v --timeout 240 --timeout-method thread > $O/pytest_B.log 2>&1 || { tail -60 $O/pytest_B.log; exit 6; }
tail -1 $O/pytest_B.log
timeout -k 10 500 python -u -m pytest $A -m gpu -v --timeout 240 --timeout-method thread > $O/pytest_A.log 2>&1 || { tail -60 $O/pytest_A.log; exit 7; }
tail -1 $O/pytest_A.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 8; }
tail -1 $O/smoke.log
