# round 6: one-rank fused reduce + AdamW (H <= 256), wgrad256 32x4 default (H = 1024): training tests,
# A/B on the same box, kernel stats of both steps
ROOT=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $ROOT
O=$ROOT/gpurun_out/r6h; mkdir -p $O
stop() { rc=$1; [ $rc -eq 124 -o $rc -eq 137 -o $rc -eq 134 -o $rc -eq 139 ] && { echo "GPU step ended rc=$rc: stopping"; exit $rc; }; [ $rc -ne 0 ] && echo "step rc=$rc"; }
timeout -k 10 600 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_train_gpu.py > $O/train_tests.log 2>&1; stop $?
tail -1 $O/train_tests.log; grep -E "FAIL|Error" $O/train_tests.log | head -20
for v in 0 1 0 1; do
  ROUTEST_FUSED_ADAMW=$v timeout -k 10 180 python -u bench/train_bench.py --hidden 256 --batch 65536 --steps 200 --warmup 20 --modes fused,graph > $O/train256_f$v.json 2>$O/train256_f$v.err; stop $?
  echo "fused_adamw=$v"; python3 -c "
import json,sys
for l in open('$O/train256_f$v.json'):
    l=l.strip()
    if l.startswith('{'):
        d=json.loads(l); print({k: (v.get('ms_per_step'), v.get('samples_per_s')) for k,v in d['results'].items()})
"
done
for c in 32x4 64x2; do
  ROUTEST_WGRAD256_CFG=$c timeout -k 10 180 python -u bench/train_bench.py --hidden 1024 --batch 65536 --steps 50 --warmup 10 --modes fused,graph > $O/train1024_$c.json 2>$O/train1024_$c.err; stop $?
  echo "cfg=$c"; tail -1 $O/train1024_$c.json | cut -c1-600
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/ks256 -o k --output-format csv -- python3 $ROOT/bench/train_bench.py --hidden 256 --batch 65536 --steps 100 --warmup 10 --modes fused > $O/ks256.log 2>&1; echo "ks256 rc=$?"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/ks1024 -o k --output-format csv -- python3 $ROOT/bench/train_bench.py --hidden 1024 --batch 65536 --steps 30 --warmup 5 --modes fused > $O/ks1024.log 2>&1; echo "ks1024 rc=$?"
ls $O/ks256 $O/ks1024
echo done
