# round 5 final (after the 16-byte GEMM epilogue stores): whole GPU suite (three parts), smoke, 2-rank shared rehearsal and the
# bench line, all with the round-end code
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
export TMPDIR=/tmp
O=$ROOT/gpurun_out/r5zu; mkdir -p $O
stop() { rc=$1; [ $rc -eq 124 -o $rc -eq 137 -o $rc -eq 134 -o $rc -eq 139 ] && { echo "GPU step ended rc=$rc: stopping"; exit $rc; }; [ $rc -ne 0 ] && echo "step rc=$rc"; }
A="tests/test_astar_gpu.py tests/test_bench_contract_gpu.py tests/test_cch_gpu.py tests/test_collective_probe_gpu.py tests/test_comm_gpu.py"
B="tests/test_eta_kernel_gpu.py tests/test_frontend_gpu.py tests/test_gcn_gpu.py tests/test_gcn_train_gpu.py tests/test_mlp_big_gpu.py tests/test_multigpu.py tests/test_multirank_gpu.py"
C="tests"; for f in $A $B; do C="$C --ignore=$f"; done
timeout -k 10 420 python -u -m pytest $C -m gpu -v --timeout 240 --timeout-method thread > $O/pytest_C.log 2>&1; stop $?
tail -1 $O/pytest_C.log
timeout -k 10 300 python -u -m pytest $B -m gpu -v --timeout 240 --timeout-method thread > $O/pytest_B.log 2>&1; stop $?
tail -1 $O/pytest_B.log
timeout -k 10 400 python -u -m pytest $A -m gpu -v --timeout 240 --timeout-method thread > $O/pytest_A.log 2>&1; stop $?
tail -1 $O/pytest_A.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1; stop $?
tail -1 $O/smoke.log
timeout -k 10 300 env ROUTEST_BENCH_SHARE_GPU=1 python bench.py --gpus 2 --steps 10 --warmup 3 --p50 0 > $O/bench_share2.log 2>&1; stop $?
grep -o '"schema_problems": \[[^]]*\]' $O/bench_share2.log
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1; stop $?
tail -1 $O/bench.log | cut -c1-200
