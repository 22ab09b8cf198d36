# round 6: wide-trainer activation rows padded to whole 128-byte lines (H + 64): tests, A/B, stats
ROOT=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $ROOT
O=$ROOT/gpurun_out/r6x; mkdir -p $O
stop() { rc=$1; [ $rc -eq 124 -o $rc -eq 137 -o $rc -eq 134 -o $rc -eq 139 ] && { echo "GPU step ended rc=$rc: stopping"; exit $rc; }; [ $rc -ne 0 ] && echo "step rc=$rc"; }
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_train_gpu.py -k "wide or dw1" > $O/train_tests.log 2>&1; stop $?
tail -1 $O/train_tests.log
for v in 1 0 1 0; do
  ROUTEST_BIG_ROW_PAD=$v timeout -k 10 180 python -u bench/train_bench.py --hidden 1024 --batch 65536 --steps 50 --warmup 10 --modes fused,graph > $O/train1024_pad$v.json 2>$O/train1024_pad$v.err; stop $?
  echo "pad=$v $(tail -1 $O/train1024_pad$v.json | cut -c150-330)"
done
for v in 1 0; do
  ROUTEST_BIG_ROW_PAD=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/ks_pad$v -o k --output-format csv -- python3 $ROOT/bench/train_bench.py --hidden 1024 --batch 65536 --steps 30 --warmup 5 --modes fused > $O/ks_pad$v.log 2>&1; echo "ks pad=$v rc=$?"
  python3 -c "
import csv
for r in list(csv.DictReader(open('$O/ks_pad$v/k_kernel_stats.csv')))[:8]: print('  ', round(float(r['AverageNs'])/1000,2), r['Name'][:60])
"
done
echo done
