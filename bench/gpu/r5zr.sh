# round 5: persistent wide GEMM with tile origins hoisted out of the load issue (second try of r5zr)
# time vs K for modes 1 and 2, H = 1024 trainer A/B
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r5zr; mkdir -p $O
stop() { rc=$1; [ $rc -eq 124 -o $rc -eq 137 -o $rc -eq 134 -o $rc -eq 139 ] && { echo "GPU step ended rc=$rc: stopping"; exit $rc; }; [ $rc -ne 0 ] && echo "step rc=$rc"; }
timeout -k 10 240 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_mlp_big_gpu.py -k "phase_pipeline" > $O/tests_gemm.log 2>&1; rc=$?; tail -3 $O/tests_gemm.log; stop $rc; [ $rc -ne 0 ] && exit $rc
for p in 2 1; do
  for K in 1024 4096; do
    ROUTEST_GEMM_PIPE=$p timeout -k 10 120 python -u bench/gemm_probe.py --k $K --iters 30 > $O/k${K}_pipe$p.json 2>$O/k${K}_pipe$p.err; stop $?
    echo "pipe=$p $(cat $O/k${K}_pipe$p.json)"
  done
done
for p in 2 1; do
  ROUTEST_GEMM_PIPE=$p timeout -k 10 180 python -u bench/train_bench.py --hidden 1024 --batch 65536 --steps 30 --warmup 5 --modes fused > $O/train1024_pipe$p.json 2>$O/train1024_pipe$p.err; stop $?
  tail -1 $O/train1024_pipe$p.json | cut -c1-300
done
echo done
