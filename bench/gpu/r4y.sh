# round 4: rehearsal of the driver's multi-rank bench path — bench.py --gpus 2 with every section on, both ranks on GPU 0
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
export TMPDIR=/tmp
O=$ROOT/gpurun_out/r4y; mkdir -p $O
ROUTEST_BENCH_SHARE_GPU=1 timeout -k 10 900 python -u bench.py --gpus 2 > $O/bench2.log 2>&1 || { tail -40 $O/bench2.log; exit 2; }
tail -1 $O/bench2.log | cut -c1-600
