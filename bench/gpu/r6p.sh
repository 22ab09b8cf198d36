# round 6 final, part 2: smoke, 2-rank shared rehearsals (clean, and with a fault injected into one
# rank's training section) and the default bench line
ROOT=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $ROOT
O=$ROOT/gpurun_out/r6p; mkdir -p $O
stop() { rc=$1; [ $rc -eq 124 -o $rc -eq 137 -o $rc -eq 134 -o $rc -eq 139 ] && { echo "GPU step ended rc=$rc: stopping"; exit $rc; }; [ $rc -ne 0 ] && echo "step rc=$rc"; }
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1; stop $?
tail -1 $O/smoke.log
timeout -k 10 300 env ROUTEST_BENCH_SHARE_GPU=1 python bench.py --gpus 2 --steps 10 --warmup 3 --p50 0 > $O/bench_share2.log 2>&1; stop $?
grep -o '"schema_problems": \[[^]]*\]' $O/bench_share2.log
timeout -k 10 300 env ROUTEST_BENCH_SHARE_GPU=1 ROUTEST_FAULT=bench_raise@train:1 python bench.py --gpus 2 --steps 10 --warmup 3 --p50 0 > $O/bench_share2_fault.log 2>&1; stop $?
grep -o '"schema_problems": \[[^]]*\]' $O/bench_share2_fault.log
timeout -k 10 500 python -u bench.py > $O/bench.log 2>&1; stop $?
tail -1 $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['route_optimizer']; print(d['value'], d['p50_predict_ms'], d['dp_training']['ms_per_step'], d['dp_training'].get('launch'), d['dp_training'].get('launch_probe_ms'), d['dp_training_large_batch']['ms_per_step'], r.get('context_customize_gpu_ms'), {k: (r[k]['req_per_s'], r[k]['p50_ms'], r[k]['p99_ms'], r[k]['stage_ms_per_flush'].get('persist'), r[k].get('record_bytes_per_row')) for k in ('http','http_f02') if k in r}, d['schema_problems'])"
echo done
