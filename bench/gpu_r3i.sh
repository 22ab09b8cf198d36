# round 3 (re-entry): validate HEAD — full GPU suite, smoke, headline bench, training + A* numbers
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r3i; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 2; }
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 3; }
tail -1 $O/bench.log
for B in 65536 1048576; do
  timeout -k 10 120 python -u bench/train_bench.py --hidden 256 --batch $B --steps 30 --warmup 5 --modes fused > $O/tb_$B.log 2>&1 || { tail -20 $O/tb_$B.log; exit 4; }
  echo "B=$B $(tail -1 $O/tb_$B.log)" | tee -a $O/train.jsonl
done
timeout -k 10 300 python -u bench/route_bench.py > $O/route_bench.log 2>&1 || { tail -30 $O/route_bench.log; exit 5; }
tail -1 $O/route_bench.log
timeout -k 10 600 python -u bench/astar_ab.py > $O/astar_ab.log 2>&1 || { tail -20 $O/astar_ab.log; exit 6; }
grep config $O/astar_ab.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/train1m -o train --output-format csv -- python3 $ROOT/bench/train_bench.py --hidden 256 --batch 1048576 --steps 10 --warmup 3 --modes fused > $O/train1m.log 2>&1 || exit 31
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/route -o route --output-format csv -- python3 $ROOT/bench/route_bench.py > $O/route_prof.log 2>&1 || exit 32
echo done
