# round 4: branch-free db2 in train_bwd_kernel (+ one branch less in the forward) — segment timing, steps, gradient tests
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
export TMPDIR=/tmp
O=$ROOT/gpurun_out/r4ak; mkdir -p $O
ROUTEST_TRAIN_BWD_PROF=1 timeout -k 10 150 python3 bench/train_bench.py --hidden 256 --batch 65536 --steps 3 --warmup 2 --modes fused > $O/p64k.log 2>&1 || { tail -20 $O/p64k.log; exit 3; }
grep "train_bwd prof" $O/p64k.log | tail -1
timeout -k 10 150 python3 bench/train_bench.py --hidden 256 --batch 65536 --steps 300 --warmup 30 --modes fused > $O/t64k.log 2>&1 || { tail -20 $O/t64k.log; exit 4; }
tail -1 $O/t64k.log | cut -c1-300
timeout -k 10 150 python3 bench/train_bench.py --hidden 256 --batch 1048576 --steps 40 --warmup 5 --modes fused > $O/t1m.log 2>&1 || { tail -20 $O/t1m.log; exit 5; }
tail -1 $O/t1m.log | cut -c1-300
timeout -k 10 300 python -u -m pytest tests/test_train_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 6; }
tail -1 $O/pytest.log
cd /tmp
timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/prof -o train --output-format csv -- python3 $ROOT/bench/train_bench.py --hidden 256 --batch 65536 --steps 30 --warmup 5 --modes fused > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 7; }
echo prof ok
