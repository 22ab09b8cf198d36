# round 6: route flush collect window from the oldest queued job vs from the wake-up (A/B, route
# sections only), with the GPU thread's collect / handoff waits
ROOT=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $ROOT
O=$ROOT/gpurun_out/r6r; mkdir -p $O
stop() { rc=$1; [ $rc -eq 124 -o $rc -eq 137 -o $rc -eq 134 -o $rc -eq 139 ] && { echo "GPU step ended rc=$rc: stopping"; exit $rc; }; [ $rc -ne 0 ] && echo "step rc=$rc"; }
i=0
for m in oldest wake oldest wake; do
  i=$((i+1))
  ROUTEST_ROUTE_COLLECT=$m timeout -k 10 300 python -u bench.py --steps 3 --warmup 2 --rec16-steps 0 --gcn-steps 0 --train-steps 0 --p50-requests 500 > $O/bench_${m}_$i.log 2>$O/bench_${m}_$i.err; stop $?
  echo "collect=$m"; tail -1 $O/bench_${m}_$i.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['route_optimizer']
for k in ('http','http_f02'):
    x=r[k]; s=x['stage_ms_per_flush']
    print('  ', k, round(x['req_per_s']), round(x['p50_ms'],2), round(x['p99_ms'],2), 'flushes', x['flushes'], {a: round(b,2) for a,b in s.items()})
"
done
echo done
# dz2y with three rows in flight: wide-trainer tests, step time, kernel stats
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_train_gpu.py -k "dw1 or wide" > $O/train_tests.log 2>&1; stop $?
tail -1 $O/train_tests.log
timeout -k 10 180 python -u bench/train_bench.py --hidden 1024 --batch 65536 --steps 50 --warmup 10 --modes fused,graph > $O/train1024.json 2>$O/train1024.err; stop $?
tail -1 $O/train1024.json | cut -c120-400
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/ks1024 -o k --output-format csv -- python3 $ROOT/bench/train_bench.py --hidden 1024 --batch 65536 --steps 30 --warmup 5 --modes fused > $O/ks1024.log 2>&1; echo "ks1024 rc=$?"
python3 -c "
import csv
for r in list(csv.DictReader(open('$O/ks1024/k_kernel_stats.csv')))[:8]: print(round(float(r['AverageNs'])/1000,1), r['Name'][:60])
"
echo done2
