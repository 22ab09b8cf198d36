# round 5: builder pacing sweep — 1M city (cached tail while fresh contexts build) and 100k graph
# (64 cold contexts) at 0 / 512 / 256 workgroups per piece
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r5q; mkdir -p $O
stop() { rc=$1; [ $rc -eq 124 -o $rc -eq 137 -o $rc -eq 134 -o $rc -eq 139 ] && { echo "GPU step ended rc=$rc: stopping"; exit $rc; }; [ $rc -ne 0 ] && echo "step rc=$rc"; }
for wg in 512 256; do
  ROUTEST_CCH_BUILDER_MAX_WG=$wg timeout -k 10 240 python -u bench/route_context_bench.py --nodes 1000000 --concurrency 256 --phases fresh > $O/fresh_wg$wg.jsonl 2>$O/fresh_wg$wg.err; stop $?
done
for wg in 0 512 256; do
  ROUTEST_CCH_BUILDER_MAX_WG=$wg timeout -k 10 200 python -u bench/route_context_bench.py --phases single,cycle64 > $O/cyc_wg$wg.jsonl 2>$O/cyc_wg$wg.err; stop $?
done
echo done
