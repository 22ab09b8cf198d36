# round 6: persistent work-queue tail of the CCH basic phase — bit-identity tests, A/B 100k and 1M
ROOT=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $ROOT
O=$ROOT/gpurun_out/r6m; mkdir -p $O
stop() { rc=$1; [ $rc -eq 124 -o $rc -eq 137 -o $rc -eq 134 -o $rc -eq 139 ] && { echo "GPU step ended rc=$rc: stopping"; exit $rc; }; [ $rc -ne 0 ] && echo "step rc=$rc"; }
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_cch_gpu.py tests/test_cch_async_gpu.py > $O/cch_tests.log 2>&1; stop $?
tail -1 $O/cch_tests.log; grep -E "FAIL|Error|cch\]" $O/cch_tests.log | head -20
for t in 4096 0 4096 0; do
  ROUTEST_CCH_TAIL=$t timeout -k 10 240 python -u bench/cch_customize_bench.py --nodes 100000 --contexts 6 --check > $O/cust100k_tail$t.jsonl 2>$O/cust100k_tail$t.err; stop $?
  echo "tail=$t"; python3 -c "
import json
for l in open('$O/cust100k_tail$t.jsonl'):
    d=json.loads(l)
    if d.get('stage')=='setup': print('  tail levels', d.get('basic_tail_levels'), 'max_height', d.get('max_height'))
    if d.get('stage')=='context': print('  ', d.get('customize_ms'), d.get('basic_ms'), d.get('perfect_ms'), d.get('prune_ms'))
    if d.get('stage')=='summary': print('  summary', d)
"
done
for t in 4096 0; do
  ROUTEST_CCH_TAIL=$t timeout -k 10 400 python -u bench/cch_customize_bench.py --nodes 1000000 --contexts 3 > $O/cust1m_tail$t.jsonl 2>$O/cust1m_tail$t.err; stop $?
  echo "1M tail=$t"; python3 -c "
import json
for l in open('$O/cust1m_tail$t.jsonl'):
    d=json.loads(l)
    if d.get('stage')=='setup': print('  tail levels', d.get('basic_tail_levels'), 'max_height', d.get('max_height'))
    if d.get('stage')=='context': print('  ', d.get('customize_ms'), d.get('basic_ms'), d.get('perfect_ms'), d.get('prune_ms'))
"
done
echo done
