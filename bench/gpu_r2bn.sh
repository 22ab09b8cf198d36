# 4-rank shared-GPU rehearsal of bench.py (self-launched ranks; one-shot DP probe at 4 ranks)
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r2bn; mkdir -p $O
ROUTEST_BENCH_SHARE_GPU=1 timeout -k 10 400 python -u bench.py --gpus 4 --steps 10 --warmup 3 --p50 0 --batch 4194304 > $O/bench4.log 2>&1 || exit 1
echo done
