# GCN: batched CSR gathers (index/weight loads, then feature rows, RB=8 in flight) — tests, bench, stats
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r2al; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gcn_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
for i in 1 2 3; do
timeout -k 10 200 python -u bench/gcn_bench.py --steps 200 --warmup 20 --mode replicate >> $O/gcn.log 2>&1 || exit 2
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o gcn --output-format csv -- python3 $ROOT/bench/gcn_bench.py --steps 20 --warmup 3 --mode replicate > $O/prof.log 2>&1 || exit 5
echo done
