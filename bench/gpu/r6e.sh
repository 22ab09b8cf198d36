# round 6: route service copies on the flush's own queue (qcopy) + restored watchdog assertions;
# wgrad256 as a 4-stage ring of 32-deep tiles (numerics, trainer A/B, kernel stats); bench line
ROOT=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $ROOT
O=$ROOT/gpurun_out/r6e; mkdir -p $O
stop() { rc=$1; [ $rc -eq 124 -o $rc -eq 137 -o $rc -eq 134 -o $rc -eq 139 ] && { echo "GPU step ended rc=$rc: stopping"; exit $rc; }; [ $rc -ne 0 ] && echo "step rc=$rc"; }
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_train_gpu.py -k "wgrad" > $O/wgrad_tests.log 2>&1; stop $?
tail -1 $O/wgrad_tests.log
for v in 0 1; do
  ROUTEST_WGRAD256=$v timeout -k 10 180 python -u bench/train_bench.py --hidden 1024 --batch 65536 --steps 50 --warmup 10 --modes fused > $O/train1024_wg$v.json 2>$O/train1024_wg$v.err; stop $?
  tail -1 $O/train1024_wg$v.json | cut -c150-300
done
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/t1k -o train --output-format csv -- python3 bench/train_bench.py --hidden 1024 --batch 65536 --steps 30 --warmup 5 --modes fused > $O/t1k.log 2>&1; stop $?
timeout -k 10 600 python -u -m pytest -v --timeout 240 --timeout-method thread tests/test_native_lifecycle_gpu.py tests/test_frontend_gpu.py tests/test_native_server_gpu.py tests/test_route_batcher_gpu.py tests/test_cch_async_gpu.py -s > $O/route_tests.log 2>&1; stop $?
grep -E "passed|failed" $O/route_tests.log | tail -2
grep -E "^\[route|^\[predict" $O/route_tests.log | head -30
timeout -k 10 500 python -u bench.py > $O/bench.log 2>&1; stop $?
tail -1 $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['route_optimizer']; print(d['value'], d['p50_predict_ms'], d['dp_training']['ms_per_step'], r.get('context_customize_gpu_ms'), {k: (r[k]['req_per_s'], r[k]['p99_ms'], r[k]['stage_ms_per_flush']) for k in ('http','http_f02') if k in r}, d['schema_problems'])"
