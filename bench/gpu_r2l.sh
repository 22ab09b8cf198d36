# training: wgrad rows-per-stage (bytes in flight) x dW2 n-split A/B
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=gpurun_out/r2l; mkdir -p $O
for kb in 32 64 128; do
  for ns in 2 3; do
    ROUTEST_WGRAD_KB=$kb ROUTEST_WGRAD_NSPLIT=$ns timeout -k 10 120 python -u bench/train_bench.py --steps 200 --warmup 20 --modes fused > $O/train_kb${kb}_ns$ns.log 2>&1 || exit 2
  done
done
cd /tmp && export TMPDIR=/tmp
ROUTEST_WGRAD_KB=64 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $ROOT/$O/prof64 -o train --output-format csv -- python3 $ROOT/bench/train_bench.py --steps 20 --warmup 5 --modes fused > $ROOT/$O/prof64.log 2>&1 || exit 4
ROUTEST_WGRAD_KB=128 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $ROOT/$O/prof128 -o train --output-format csv -- python3 $ROOT/bench/train_bench.py --steps 20 --warmup 5 --modes fused > $ROOT/$O/prof128.log 2>&1 || exit 5
echo done
