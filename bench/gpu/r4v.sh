# round 4: the whole GPU suite in three parts (A|B|C by argument) + smoke after C
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
export TMPDIR=/tmp
PART=$1
O=$ROOT/gpurun_out/r4v; mkdir -p $O
A="tests/test_astar_gpu.py tests/test_bench_contract_gpu.py tests/test_cch_gpu.py tests/test_collective_probe_gpu.py tests/test_comm_gpu.py"
B="tests/test_eta_kernel_gpu.py tests/test_frontend_gpu.py tests/test_gcn_gpu.py tests/test_gcn_train_gpu.py tests/test_mlp_big_gpu.py tests/test_multigpu.py tests/test_multirank_gpu.py"
if [ "$PART" = A ]; then SEL="$A"; elif [ "$PART" = B ]; then SEL="$B"; else
  SEL="tests"; for f in $A $B; do SEL="$SEL --ignore=$f"; done; fi
timeout -k 10 1100 python -u -m pytest $SEL -m gpu -v --timeout 240 --timeout-method thread > $O/pytest_$PART.log 2>&1 || { tail -80 $O/pytest_$PART.log; exit 2; }
tail -1 $O/pytest_$PART.log
if [ "$PART" = C ]; then
  timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 3; }
  tail -1 $O/smoke.log
fi
