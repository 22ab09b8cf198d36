# stress the one-shot collectives (fused stage+signal): 2 and 4 ranks sharing GPU 0
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r2az; mkdir -p $O
timeout -k 10 300 python -u tools/stress_oneshot.py 2 3000 > $O/stress2.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/stress_oneshot.py 4 2000 > $O/stress4.log 2>&1 || exit 2
echo done
