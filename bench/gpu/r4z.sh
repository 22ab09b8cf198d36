# round 4: eager vs HIP-graph training step at 64k / 1M rows (H=256) and H=1024
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
export TMPDIR=/tmp
O=$ROOT/gpurun_out/r4z; mkdir -p $O
timeout -k 10 200 python3 bench/train_bench.py --hidden 256 --batch 65536 --steps 300 --warmup 30 --modes fused,graph > $O/t64k.log 2>&1 || { tail -20 $O/t64k.log; exit 2; }
tail -1 $O/t64k.log | cut -c1-500
timeout -k 10 200 python3 bench/train_bench.py --hidden 256 --batch 1048576 --steps 40 --warmup 5 --modes fused,graph > $O/t1m.log 2>&1 || { tail -20 $O/t1m.log; exit 3; }
tail -1 $O/t1m.log | cut -c1-500
timeout -k 10 200 python3 bench/train_bench.py --hidden 1024 --batch 65536 --steps 40 --warmup 5 --modes fused,graph > $O/t1k.log 2>&1 || { tail -20 $O/t1k.log; exit 4; }
tail -1 $O/t1k.log | cut -c1-500
