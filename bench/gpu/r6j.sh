# round 6: dW1 in the dgrad epilogue (H = 1024) tests + A/B; host CPU quota vs the http_f02 tail
ROOT=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $ROOT
O=$ROOT/gpurun_out/r6j; mkdir -p $O
stop() { rc=$1; [ $rc -eq 124 -o $rc -eq 137 -o $rc -eq 134 -o $rc -eq 139 ] && { echo "GPU step ended rc=$rc: stopping"; exit $rc; }; [ $rc -ne 0 ] && echo "step rc=$rc"; }
{ echo "nproc $(nproc)"; python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)))"; cat /proc/self/cgroup; for f in cpu.max cpu.stat cpu.weight; do echo "== $f"; cat /sys/fs/cgroup/$f 2>&1; done; } > $O/cgroup.txt 2>&1
cat $O/cgroup.txt | head -30
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_train_gpu.py -k "dw1 or wide" > $O/train_tests.log 2>&1; stop $?
tail -1 $O/train_tests.log; grep -E "FAIL|Error" $O/train_tests.log | head -20
for v in 1 0 1 0; do
  ROUTEST_DW1_EPILOGUE=$v timeout -k 10 180 python -u bench/train_bench.py --hidden 1024 --batch 65536 --steps 50 --warmup 10 --modes fused,graph > $O/train1024_e$v.json 2>$O/train1024_e$v.err; stop $?
  echo "dw1_epilogue=$v $(tail -1 $O/train1024_e$v.json | cut -c120-400)"
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/ks1024 -o k --output-format csv -- python3 $ROOT/bench/train_bench.py --hidden 1024 --batch 65536 --steps 30 --warmup 5 --modes fused > $O/ks1024.log 2>&1; echo "ks1024 rc=$?"
cat /sys/fs/cgroup/cpu.stat > $O/cpu_stat_before.txt 2>&1
ROUTEST_ROUTE_TRACE_MS=8 timeout -k 10 300 python -u bench.py --steps 3 --warmup 2 --rec16-steps 0 --gcn-steps 0 --train-steps 0 --p50-requests 500 > $O/bench1.log 2>$O/bench1.err; stop $?
cat /sys/fs/cgroup/cpu.stat > $O/cpu_stat_after.txt 2>&1
tail -1 $O/bench1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['route_optimizer']; print({k: (r[k]['req_per_s'], r[k]['p50_ms'], r[k]['p99_ms']) for k in ('http','http_f02') if k in r})"
paste $O/cpu_stat_before.txt $O/cpu_stat_after.txt
echo done
