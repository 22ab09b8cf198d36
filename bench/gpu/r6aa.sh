# round 6: the wide trainer's one-rank fused reduce + AdamW — bitwise test, training tests, A/B, stats
ROOT=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $ROOT
O=$ROOT/gpurun_out/r6aa; mkdir -p $O
stop() { rc=$1; [ $rc -eq 124 -o $rc -eq 137 -o $rc -eq 134 -o $rc -eq 139 ] && { echo "GPU step ended rc=$rc: stopping"; exit $rc; }; [ $rc -ne 0 ] && echo "step rc=$rc"; }
timeout -k 10 600 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_train_gpu.py > $O/train_tests.log 2>&1; stop $?
tail -1 $O/train_tests.log; grep -E "FAILED|ERROR|assert" $O/train_tests.log | head -20
for v in 1 0 1 0; do
  ROUTEST_FUSED_ADAMW=$v timeout -k 10 180 python -u bench/train_bench.py --hidden 1024 --batch 65536 --steps 50 --warmup 10 --modes fused,graph > $O/train1024_f$v.json 2>$O/train1024_f$v.err; stop $?
  echo "fused=$v $(tail -1 $O/train1024_f$v.json | cut -c150-330)"
done
timeout -k 10 120 python -u bench/train_bench.py --hidden 1024 --batch 262144 --steps 20 --warmup 5 --modes fused > $O/train1024_262k.json 2>$O/train1024_262k.err; stop $?
echo "262k $(tail -1 $O/train1024_262k.json | cut -c150-330)"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/ks1024 -o k --output-format csv -- python3 $ROOT/bench/train_bench.py --hidden 1024 --batch 65536 --steps 30 --warmup 5 --modes fused > $O/ks1024.log 2>&1; echo "ks rc=$?"
python3 -c "
import csv
for r in list(csv.DictReader(open('$O/ks1024/k_kernel_stats.csv')))[:8]: print('  ', round(float(r['AverageNs'])/1000,2), r['Name'][:60])
"
echo done
