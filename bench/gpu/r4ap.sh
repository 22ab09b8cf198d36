# round 4: gemm256_kernel with both k-steps' fragments read up front — probe, H=1024 trainer, wide-MLP tests
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
export TMPDIR=/tmp
O=$ROOT/gpurun_out/r4ap; mkdir -p $O
timeout -k 10 120 python -u -m pytest tests/test_mlp_big_gpu.py -x -q --timeout 100 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 2; }
tail -1 $O/pytest.log
timeout -k 10 120 python3 bench/gemm_probe.py > $O/gemm.json 2>$O/gemm.err || { tail -20 $O/gemm.err; exit 3; }
cat $O/gemm.json
timeout -k 10 150 python3 bench/train_bench.py --hidden 1024 --batch 65536 --steps 40 --warmup 5 --modes fused > $O/t1k.log 2>&1 || { tail -20 $O/t1k.log; exit 4; }
tail -1 $O/t1k.log | cut -c1-300
