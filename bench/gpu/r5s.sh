# round 5: default builder pacing check (1M fresh), CCH tests, and the HIP-graph probe of the
# customization launch sequence (100k and 1M)
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r5s; mkdir -p $O
stop() { rc=$1; [ $rc -eq 124 -o $rc -eq 137 -o $rc -eq 134 -o $rc -eq 139 ] && { echo "GPU step ended rc=$rc: stopping"; exit $rc; }; [ $rc -ne 0 ] && echo "step rc=$rc"; }
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_cch_gpu.py tests/test_cch_async_gpu.py > $O/tests.log 2>&1; stop $?
ROUTEST_CCH_GRAPH_PROBE=10 timeout -k 10 200 python -u bench/cch_customize_bench.py --contexts 2 > $O/probe100k.log 2>&1; stop $?
ROUTEST_CCH_GRAPH_PROBE=3 timeout -k 10 240 python -u bench/cch_customize_bench.py --nodes 1000000 --contexts 2 > $O/probe1m.log 2>&1; stop $?
timeout -k 10 240 python -u bench/route_context_bench.py --nodes 1000000 --concurrency 256 --phases fresh > $O/fresh_default.jsonl 2>$O/fresh_default.err; stop $?
echo done
