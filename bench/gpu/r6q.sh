# round 6: where the config-5 bulk step (10k requests, CCH) spends its 24 ms — kernel trace + stats
ROOT=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $ROOT
O=$ROOT/gpurun_out/r6q; mkdir -p $O
timeout -k 10 300 python -u bench/route_bench.py --steps 10 --warmup 2 > $O/route_bench.json 2>$O/route_bench.err; echo "rc=$?"; tail -1 $O/route_bench.json | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ks -o k --output-format csv -- python3 $ROOT/bench/route_bench.py --steps 10 --warmup 2 > $O/ks.log 2>&1; echo "ks rc=$?"
python3 -c "
import csv
for r in list(csv.DictReader(open('$O/ks/k_kernel_stats.csv')))[:25]: print(r['Calls'], round(float(r['TotalDurationNs'])/1e6,2), round(float(r['AverageNs'])/1000,1), r['Name'][:90])
"
echo done
