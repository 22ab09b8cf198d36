# stress: 2-runner micro-batcher on one GPU (8 rounds x 6000 concurrent requests)
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r2ax; mkdir -p $O
timeout -k 10 400 python -u tools/stress_batcher_two_runners.py 40 > $O/stress.log 2>&1 || exit 1
echo done
