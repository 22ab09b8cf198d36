# round 4 final check: trainer timing with the v_dot2 db2, then the whole GPU suite (three parts) and smoke
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
export TMPDIR=/tmp
O=$ROOT/gpurun_out/r4an; mkdir -p $O
ROUTEST_TRAIN_BWD_PROF=1 timeout -k 10 150 python3 bench/train_bench.py --hidden 256 --batch 65536 --steps 3 --warmup 2 --modes fused > $O/p64k.log 2>&1 || { tail -20 $O/p64k.log; exit 2; }
grep "train_bwd prof" $O/p64k.log | tail -1
timeout -k 10 150 python3 bench/train_bench.py --hidden 256 --batch 65536 --steps 300 --warmup 30 --modes fused > $O/t64k.log 2>&1 || { tail -20 $O/t64k.log; exit 3; }
tail -1 $O/t64k.log | cut -c1-300
timeout -k 10 150 python3 bench/train_bench.py --hidden 256 --batch 1048576 --steps 40 --warmup 5 --modes fused > $O/t1m.log 2>&1 || { tail -20 $O/t1m.log; exit 4; }
tail -1 $O/t1m.log | cut -c1-300
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
