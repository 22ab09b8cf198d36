# round 5: kernel stats of the H = 1024 training step with the round-end wide GEMM (phase pipeline +
# 16-byte epilogue stores)
ROOT=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $ROOT
O=$ROOT/gpurun_out/r5zv; mkdir -p $O
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/t1k -o train --output-format csv -- python3 bench/train_bench.py --hidden 1024 --batch 65536 --steps 30 --warmup 5 --modes fused > $O/t1k.log 2>&1 || { echo "train stats failed rc=$?"; exit 1; }
timeout -k 10 180 python -u bench/train_bench.py --hidden 1024 --batch 65536 --steps 50 --warmup 10 --modes fused > $O/train1024_b65536.json 2>$O/train1024.err || exit 1
timeout -k 10 180 python -u bench/train_bench.py --hidden 1024 --batch 262144 --steps 20 --warmup 5 --modes fused > $O/train1024_b262144.json 2>>$O/train1024.err || exit 1
tail -1 $O/train1024_b65536.json | cut -c1-250; tail -1 $O/train1024_b262144.json | cut -c1-250
echo done
