# round 6: http_f02 tail — which stage outlasts 8 ms (route-service stage trace), two runs
ROOT=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $ROOT
O=$ROOT/gpurun_out/r6i; mkdir -p $O
stop() { rc=$1; [ $rc -eq 124 -o $rc -eq 137 -o $rc -eq 134 -o $rc -eq 139 ] && { echo "GPU step ended rc=$rc: stopping"; exit $rc; }; [ $rc -ne 0 ] && echo "step rc=$rc"; }
for i in 1 2; do
  ROUTEST_ROUTE_TRACE_MS=8 timeout -k 10 300 python -u bench.py --steps 3 --warmup 2 --rec16-steps 0 --gcn-steps 0 --train-steps 0 --p50-requests 500 > $O/bench$i.log 2>$O/bench$i.err; stop $?
  tail -1 $O/bench$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['route_optimizer']; print({k: (r[k]['req_per_s'], r[k]['p50_ms'], r[k]['p99_ms'], r[k]['stage_ms_per_flush']) for k in ('http','http_f02') if k in r})"
  grep -c "took" $O/bench$i.err; grep "took" $O/bench$i.err | awk '{print $5}' | sort | uniq -c
done
echo done
