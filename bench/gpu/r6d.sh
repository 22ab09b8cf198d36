# round 6: wgrad256 (H = 1024 dW2 on 256x256 output tiles) numerics + trainer A/B + kernel stats;
# watchdog rehearsal with the route / predict trace (ROUTEST_ROUTE_TRACE_MS)
ROOT=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $ROOT
O=$ROOT/gpurun_out/r6d; mkdir -p $O
stop() { rc=$1; [ $rc -eq 124 -o $rc -eq 137 -o $rc -eq 134 -o $rc -eq 139 ] && { echo "GPU step ended rc=$rc: stopping"; exit $rc; }; [ $rc -ne 0 ] && echo "step rc=$rc"; }
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_train_gpu.py -k "wgrad" > $O/wgrad_tests.log 2>&1; stop $?
tail -3 $O/wgrad_tests.log
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_mlp_big_gpu.py tests/test_train_gpu.py > $O/train_tests.log 2>&1; stop $?
tail -3 $O/train_tests.log
for v in 0 1; do
  ROUTEST_WGRAD256=$v timeout -k 10 180 python -u bench/train_bench.py --hidden 1024 --batch 65536 --steps 50 --warmup 10 --modes fused > $O/train1024_wg$v.json 2>$O/train1024_wg$v.err; stop $?
  tail -1 $O/train1024_wg$v.json | cut -c1-300
done
ROUTEST_WGRAD256=1 timeout -k 10 180 python -u bench/train_bench.py --hidden 1024 --batch 262144 --steps 20 --warmup 5 --modes fused > $O/train1024_b262k.json 2>>$O/train1024_wg1.err; stop $?
tail -1 $O/train1024_b262k.json | cut -c1-300
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/t1k -o train --output-format csv -- python3 bench/train_bench.py --hidden 1024 --batch 65536 --steps 30 --warmup 5 --modes fused > $O/t1k.log 2>&1; stop $?
export GPU_MAX_HW_QUEUES=32 ROUTEST_GPU_DEADLINE_MS=100 ROUTEST_ROUTE_DEADLINE_MS=300 ROUTEST_PERSIST_IDLE_MS=0 ROUTEST_QUARANTINE_PROBE_MS=60000 ROUTEST_HANG_ARM=1 ROUTEST_ROUTE_TRACE_MS=20
timeout -k 10 200 python3 -u tests/_watchdog_child.py > $O/child_trace.log 2>&1; stop $?
grep -c "route slot\|predict slot" $O/child_trace.log
tail -c 1200 $O/child_trace.log
unset GPU_MAX_HW_QUEUES ROUTEST_GPU_DEADLINE_MS ROUTEST_ROUTE_DEADLINE_MS ROUTEST_PERSIST_IDLE_MS ROUTEST_QUARANTINE_PROBE_MS ROUTEST_HANG_ARM ROUTEST_ROUTE_TRACE_MS
timeout -k 10 500 python -u bench.py > $O/bench.log 2>&1; stop $?
tail -1 $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['route_optimizer']; print(d['value'], d['p50_predict_ms'], d['dp_training']['ms_per_step'], r.get('context_customize_gpu_ms'), {k: (r[k]['req_per_s'], r[k]['p99_ms'], r[k]['stage_ms_per_flush']) for k in ('http','http_f02') if k in r}, d['schema_problems'])"
