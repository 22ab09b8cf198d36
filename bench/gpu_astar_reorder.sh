# A* node renumbering A/B (Morton vs caller ids) + exactness tests (run on the GPU box)
cd $GRAFT_REPO_ROOT
O=gpurun_out/areorder; mkdir -p $O
timeout -k 10 240 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_astar_gpu.py > $O/tests.log 2>&1 || exit 1
for r in 1 0 1; do
  ROUTEST_ASTAR_REORDER=$r timeout -k 10 150 python -u bench/astar_tail.py >> $O/tail_$r.log 2>&1 || exit 1
done
ROUTEST_ASTAR_REORDER=1 timeout -k 10 200 python -u bench/route_bench.py > $O/route_1.log 2>&1 || exit 1
echo done
