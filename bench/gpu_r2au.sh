# A* wave stage: target landmark row in registers (HU=0, 4 waves/SIMD) vs LDS with HU row loads per round
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r2au; mkdir -p $O
ROUTEST_ASTAR_WAVE_HU=2 timeout -k 10 300 python -u -m pytest tests/test_astar_gpu.py -x -q --timeout 250 --timeout-method thread > $O/pytest_hu2.log 2>&1 || exit 1
for r in 1 2; do
for hu in 0 1 2 4; do
  echo "HU=$hu" >> $O/route.log
  ROUTEST_ASTAR_WAVE_HU=$hu timeout -k 10 200 python -u bench/route_bench.py --steps 5 --warmup 1 >> $O/route.log 2>&1 || exit 2
done
done
echo done
