# round 5: 16-byte epilogue stores of the 256 x 256 wide GEMM (lane-pair exchange) vs 8-byte stores
# (ROUTEST_GEMM_ST16 A/B), both on the phase-pipelined K loop; tests first
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r5zt; mkdir -p $O
stop() { rc=$1; [ $rc -eq 124 -o $rc -eq 137 -o $rc -eq 134 -o $rc -eq 139 ] && { echo "GPU step ended rc=$rc: stopping"; exit $rc; }; [ $rc -ne 0 ] && echo "step rc=$rc"; }
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_mlp_big_gpu.py > $O/tests_big.log 2>&1; rc=$?; tail -2 $O/tests_big.log; stop $rc; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_train_gpu.py -k "wide or 512 or 1024" > $O/tests_train.log 2>&1; rc=$?; tail -2 $O/tests_train.log; stop $rc; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for st in 1 0; do
    ROUTEST_GEMM_ST16=$st timeout -k 10 120 python -u bench/gemm_probe.py --iters 50 > $O/st${st}_rep$rep.json 2>$O/st${st}_rep$rep.err; stop $?
    echo "st16=$st $(cat $O/st${st}_rep$rep.json)"
  done
done
for st in 1 0; do
  ROUTEST_GEMM_ST16=$st timeout -k 10 180 python -u bench/train_bench.py --hidden 1024 --batch 65536 --steps 30 --warmup 5 --modes fused > $O/train1024_st$st.json 2>$O/train1024_st$st.err; stop $?
  echo "st16=$st $(tail -1 $O/train1024_st$st.json | cut -c1-250)"
done
echo done
