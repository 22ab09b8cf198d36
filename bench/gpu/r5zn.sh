# round 5: phase-pipelined wide GEMM (gemm256p_kernel) — bitwise vs the drain loop, the H = 1024 / 512
# trainer tests, then the GEMM probe and the H = 1024 training step with each K loop
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r5zn; mkdir -p $O
stop() { rc=$1; [ $rc -eq 124 -o $rc -eq 137 -o $rc -eq 134 -o $rc -eq 139 ] && { echo "GPU step ended rc=$rc: stopping"; exit $rc; }; [ $rc -ne 0 ] && echo "step rc=$rc"; }
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_mlp_big_gpu.py > $O/tests_big.log 2>&1; rc=$?; tail -5 $O/tests_big.log; stop $rc; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_train_gpu.py -k "wide or 512 or 1024" > $O/tests_train.log 2>&1; rc=$?; tail -3 $O/tests_train.log; stop $rc
for p in 0 1; do
  ROUTEST_GEMM_PIPE=$p timeout -k 10 120 python -u bench/gemm_probe.py --iters 50 > $O/gemm_pipe$p.json 2>$O/gemm_pipe$p.err; stop $?
  cat $O/gemm_pipe$p.json
done
for p in 0 1; do
  for B in 65536 262144; do
    ROUTEST_GEMM_PIPE=$p timeout -k 10 180 python -u bench/train_bench.py --hidden 1024 --batch $B --steps 30 --warmup 5 --modes fused > $O/train1024_b${B}_pipe$p.json 2>$O/train1024_b${B}_pipe$p.err; stop $?
    tail -1 $O/train1024_b${B}_pipe$p.json | cut -c1-400
  done
done
echo done
