# bench.py with the GCN probe (1 GPU: replicate) — timing of the whole run
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r2y; mkdir -p $O
SECONDS=0; timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
echo "bench seconds $SECONDS" > $O/time.txt; echo done
