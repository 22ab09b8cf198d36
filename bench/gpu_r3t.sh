# round 3: wave-tier f-band pass statistics (mean near-set size per pass)
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r3t; mkdir -p $O
timeout -k 10 300 python -u bench/astar_passes.py > $O/exp.log 2>&1 || { tail -20 $O/exp.log; exit 1; }
tail -1 $O/exp.log
ROUTEST_ASTAR_COUNT_PASSES=1 timeout -k 10 300 python -u bench/astar_passes.py > $O/passes.log 2>&1 || { tail -20 $O/passes.log; exit 2; }
tail -1 $O/passes.log
