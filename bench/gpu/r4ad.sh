# round 4: train_bwd_kernel per-tile segment timing (s_memtime instrumentation build, diagnostics) at 64k and 1M rows
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
export TMPDIR=/tmp
O=$ROOT/gpurun_out/r4ad; mkdir -p $O
ROUTEST_TRAIN_BWD_PROF=1 timeout -k 10 150 python3 bench/train_bench.py --hidden 256 --batch 65536 --steps 3 --warmup 2 --modes fused > $O/p64k.log 2>&1 || { tail -20 $O/p64k.log; exit 2; }
grep "train_bwd prof" $O/p64k.log | tail -2
ROUTEST_TRAIN_BWD_PROF=1 timeout -k 10 150 python3 bench/train_bench.py --hidden 256 --batch 1048576 --steps 3 --warmup 2 --modes fused > $O/p1m.log 2>&1 || { tail -20 $O/p1m.log; exit 3; }
grep "train_bwd prof" $O/p1m.log | tail -2
