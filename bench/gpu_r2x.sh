# bench.py with the DP-training probe and per-step distribution: 1 GPU default + 2-rank shared rehearsal
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r2x; mkdir -p $O
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
export ROUTEST_BENCH_SHARE_GPU=1
timeout -k 10 300 python -u bench.py --gpus 2 --steps 5 --warmup 2 --batch 1048576 --p50 0 --train-steps 10 > $O/bench_2rank_shared.json 2> $O/bench_2rank.err || exit 2
echo done
