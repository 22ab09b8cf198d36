# round 4: pipelined wide GEMM (gemm256p) A/B + H=1024 trainer; mixed soak with per-endpoint latency
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
export TMPDIR=/tmp
O=$ROOT/gpurun_out/r4p; mkdir -p $O
timeout -k 10 120 python -u -m pytest tests/test_mlp_big_gpu.py -x -v --timeout 100 --timeout-method thread > $O/pytest_big.log 2>&1 || { tail -40 $O/pytest_big.log; exit 2; }
tail -1 $O/pytest_big.log
ROUTEST_GEMM_PIPE=0 timeout -k 10 120 python3 bench/gemm_probe.py > $O/gemm_2stage.json 2>$O/gemm_2stage.err || { tail -20 $O/gemm_2stage.err; exit 3; }
cat $O/gemm_2stage.json
timeout -k 10 120 python3 bench/gemm_probe.py > $O/gemm_pipe.json 2>$O/gemm_pipe.err || { tail -20 $O/gemm_pipe.err; exit 4; }
cat $O/gemm_pipe.json
ROUTEST_GEMM_PIPE=0 timeout -k 10 150 python3 bench/train_bench.py --hidden 1024 --batch 65536 --steps 20 --warmup 5 --modes fused > $O/train_h1024_2stage.log 2>&1 || { tail -20 $O/train_h1024_2stage.log; exit 5; }
tail -1 $O/train_h1024_2stage.log | cut -c1-400
timeout -k 10 150 python3 bench/train_bench.py --hidden 1024 --batch 65536 --steps 20 --warmup 5 --modes fused > $O/train_h1024_pipe.log 2>&1 || { tail -20 $O/train_h1024_pipe.log; exit 6; }
tail -1 $O/train_h1024_pipe.log | cut -c1-400
timeout -k 10 300 python3 tools/app_soak.py --stack --clients 128 --seconds 20 > $O/soak.log 2>&1 || { tail -20 $O/soak.log; exit 7; }
tail -1 $O/soak.log | cut -c1-3000
