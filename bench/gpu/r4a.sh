# round 4: A* multi-wave exactness (ADVICE r3 race fix) + checkpoint
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
export TMPDIR=/tmp
O=$ROOT/gpurun_out/r4a; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_astar_gpu.py -x -v --timeout 240 --timeout-method thread > $O/pytest_astar.log 2>&1 || { tail -60 $O/pytest_astar.log; exit 1; }
tail -3 $O/pytest_astar.log
