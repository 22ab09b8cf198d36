# round 3: wide-trainer (H = 1024) kernel profile at 64k / 256k rows + hipBLASLt reference on the same GEMM shapes
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
export TMPDIR=/tmp
O=$ROOT/gpurun_out/r3v; mkdir -p $O
timeout -k 10 180 python -u bench/gemm_probe.py 1024 > $O/gemm_probe.log 2>&1 || { tail -20 $O/gemm_probe.log; exit 2; }
grep '^{' $O/gemm_probe.log
for B in 65536 262144; do
  timeout -k 10 180 python -u bench/train_bench.py --hidden 1024 --batch $B --steps 20 --warmup 3 --modes fused > $O/tb_$B.log 2>&1 || { tail -20 $O/tb_$B.log; exit 3; }
  tail -1 $O/tb_$B.log
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o h1024 -- python3 bench/train_bench.py --hidden 1024 --batch 65536 --steps 10 --warmup 2 --modes fused > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 4; }
cp "$(find $O/prof -name '*kernel_stats.csv' -print -quit)" $O/h1024_64k_kernel_stats.csv
echo done
