# round 6: tiled relu bit mask (H = 1024 dW1 epilogue) A/B + kernel stats; CCH tails (basic + perfect)
# at small thresholds
ROOT=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $ROOT
O=$ROOT/gpurun_out/r6n; mkdir -p $O
stop() { rc=$1; [ $rc -eq 124 -o $rc -eq 137 -o $rc -eq 134 -o $rc -eq 139 ] && { echo "GPU step ended rc=$rc: stopping"; exit $rc; }; [ $rc -ne 0 ] && echo "step rc=$rc"; }
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_train_gpu.py -k "dw1 or wide" > $O/train_tests.log 2>&1; stop $?
tail -1 $O/train_tests.log; grep -E "FAIL|Error" $O/train_tests.log | head -20
for v in 1 0 1; do
  ROUTEST_DW1_EPILOGUE=$v timeout -k 10 180 python -u bench/train_bench.py --hidden 1024 --batch 65536 --steps 50 --warmup 10 --modes fused,graph > $O/train1024_e$v.json 2>$O/train1024_e$v.err; stop $?
  echo "dw1_epilogue=$v $(tail -1 $O/train1024_e$v.json | cut -c120-400)"
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/ks1024 -o k --output-format csv -- python3 $ROOT/bench/train_bench.py --hidden 1024 --batch 65536 --steps 30 --warmup 5 --modes fused > $O/ks1024.log 2>&1; echo "ks1024 rc=$?"
python3 -c "
import csv
for r in list(csv.DictReader(open('$O/ks1024/k_kernel_stats.csv')))[:8]: print(round(float(r['AverageNs'])/1000,1), r['Name'][:60])
"
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_cch_gpu.py > $O/cch_tests.log 2>&1; stop $?
tail -1 $O/cch_tests.log
for t in 64 512 0; do
  ROUTEST_CCH_TAIL=$t timeout -k 10 240 python -u bench/cch_customize_bench.py --nodes 100000 --contexts 4 --check > $O/cust100k_tail$t.jsonl 2>$O/cust100k_tail$t.err; stop $?
  echo "tail=$t"; python3 -c "
import json
for l in open('$O/cust100k_tail$t.jsonl'):
    d=json.loads(l)
    if d.get('stage')=='setup': print('  tail levels', d.get('basic_tail_levels'), d.get('perfect_tail_levels'))
    if d.get('stage')=='context': print('  ', d.get('customize_ms'), d.get('basic_ms'), d.get('perfect_ms'))
    if d.get('stage')=='summary': print('  bit identical', d.get('bit_identical_vs_cpu'))
"
done
echo done
