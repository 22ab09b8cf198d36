# round 6: wgrad256 with inline-asm LDS DMA (no compiler drain before the fragment reads) + raw
# barriers: numerics, probe A/B (64x2 / 32x4 / wgrad<9>), trainer A/B, PMC pass 1
ROOT=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $ROOT
O=$ROOT/gpurun_out/r6g; mkdir -p $O
stop() { rc=$1; [ $rc -eq 124 -o $rc -eq 137 -o $rc -eq 134 -o $rc -eq 139 ] && { echo "GPU step ended rc=$rc: stopping"; exit $rc; }; [ $rc -ne 0 ] && echo "step rc=$rc"; }
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_train_gpu.py -k "wgrad256" > $O/wgrad_tests.log 2>&1; stop $?
tail -1 $O/wgrad_tests.log
ROUTEST_WGRAD256_CFG=32x4 timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_train_gpu.py -k "wgrad256" > $O/wgrad_tests_32x4.log 2>&1; stop $?
tail -1 $O/wgrad_tests_32x4.log
timeout -k 10 120 python -u bench/wgrad_probe.py --iters 20 > $O/probe_64x2.jsonl 2>&1; stop $?
ROUTEST_WGRAD256_CFG=32x4 timeout -k 10 120 python -u bench/wgrad_probe.py --iters 20 --kernels wgrad256 > $O/probe_32x4.jsonl 2>&1; stop $?
grep kernel $O/probe_64x2.jsonl $O/probe_32x4.jsonl
for v in 0 1; do
  ROUTEST_WGRAD256=$v timeout -k 10 180 python -u bench/train_bench.py --hidden 1024 --batch 65536 --steps 50 --warmup 10 --modes fused > $O/train1024_wg$v.json 2>$O/train1024_wg$v.err; stop $?
  tail -1 $O/train1024_wg$v.json | cut -c150-300
done
G1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $G1 -d $O/pmc_1 -o w --output-format csv -- python3 $ROOT/bench/wgrad_probe.py --iters 5 > $O/pmc_1.log 2>&1 || { echo "pmc failed rc=$?"; exit 1; }
echo done
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_frontend_gpu.py -k "compact_records" > $O/records_test.log 2>&1; stop $?
tail -1 $O/records_test.log
timeout -k 10 500 python -u bench.py > $O/bench.log 2>&1; stop $?
tail -1 $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['route_optimizer']; print(d['value'], d['p50_predict_ms'], d['dp_training']['ms_per_step'], d['dp_training'].get('launch'), d['dp_training_large_batch']['ms_per_step'], r.get('context_customize_gpu_ms'), {k: (r[k]['req_per_s'], r[k]['p99_ms'], r[k].get('record_bytes_per_row')) for k in ('http','http_f02') if k in r}, d['schema_problems'])"
