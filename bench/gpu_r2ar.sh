# default bench at HEAD (incl. large-batch DP probe) + a kernel-trace/stats profile of the whole bench run
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r2ar; mkdir -p $O
s0=$SECONDS; timeout -k 10 400 python -u bench.py > $O/bench.log 2> $O/bench.err || exit 1; echo "bench wall $((SECONDS-s0)) s" > $O/bench_wall.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- python3 $ROOT/bench.py --steps 10 --warmup 3 --p50 0 > $O/prof.log 2>&1 || exit 2
echo done
