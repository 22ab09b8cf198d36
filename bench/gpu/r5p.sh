# round 5: pacing the background builder (wide customization levels launched in pieces of N
# workgroups) against the cached requests' tail while 1M-city contexts build; paced build exact
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r5p; mkdir -p $O
stop() { rc=$1; [ $rc -eq 124 -o $rc -eq 137 -o $rc -eq 134 -o $rc -eq 139 ] && { echo "GPU step ended rc=$rc: stopping"; exit $rc; }; [ $rc -ne 0 ] && echo "step rc=$rc"; }
timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_cch_gpu.py > $O/tests.log 2>&1; stop $?
for wg in 0 256 64; do
  ROUTEST_CCH_BUILDER_MAX_WG=$wg timeout -k 10 240 python -u bench/route_context_bench.py --nodes 1000000 --concurrency 256 --phases fresh > $O/fresh_wg$wg.jsonl 2>$O/fresh_wg$wg.err; stop $?
done
echo done
