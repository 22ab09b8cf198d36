# round 6: slab reduce variants (r6t: eight loads in flight; r6u: 32 slice lanes x 8 columns) — training tests, H = 256 / 1024 steps, stats
ROOT=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $ROOT
O=$ROOT/gpurun_out/${RUN:-r6t}; mkdir -p $O
stop() { rc=$1; [ $rc -eq 124 -o $rc -eq 137 -o $rc -eq 134 -o $rc -eq 139 ] && { echo "GPU step ended rc=$rc: stopping"; exit $rc; }; [ $rc -ne 0 ] && echo "step rc=$rc"; }
timeout -k 10 600 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_train_gpu.py > $O/train_tests.log 2>&1; stop $?
tail -1 $O/train_tests.log; grep -E "FAILED|ERROR" $O/train_tests.log | head
for i in 1 2; do
  timeout -k 10 180 python -u bench/train_bench.py --hidden 256 --batch 65536 --steps 200 --warmup 20 --modes fused,graph > $O/train256_$i.json 2>$O/train256_$i.err; stop $?
  tail -1 $O/train256_$i.json | cut -c120-400
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/ks256 -o k --output-format csv -- python3 $ROOT/bench/train_bench.py --hidden 256 --batch 65536 --steps 100 --warmup 10 --modes fused > $O/ks256.log 2>&1; echo "ks256 rc=$?"
python3 -c "
import csv
for r in list(csv.DictReader(open('$O/ks256/k_kernel_stats.csv')))[:5]: print(round(float(r['AverageNs'])/1000,2), r['Name'][:60])
"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/ks1024 -o k --output-format csv -- python3 $ROOT/bench/train_bench.py --hidden 1024 --batch 65536 --steps 30 --warmup 5 --modes fused > $O/ks1024.log 2>&1; echo "ks1024 rc=$?"
python3 -c "
import csv
for r in list(csv.DictReader(open('$O/ks1024/k_kernel_stats.csv')))[:8]: print(round(float(r['AverageNs'])/1000,2), r['Name'][:60])
"
echo done
