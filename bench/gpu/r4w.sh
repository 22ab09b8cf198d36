# round 4: bench.py with no flags (the driver's N=1 run) after the persistence / front-end / trainer work
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
export TMPDIR=/tmp
O=$ROOT/gpurun_out/r4w; mkdir -p $O
timeout -k 10 900 python -u bench.py > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 2; }
tail -1 $O/bench.log | cut -c1-400
