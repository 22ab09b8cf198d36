# round 5: (tail, head) -> arc hash in the basic finalize step: customization + tests
# on levels that do not fill the GPU: customization on the 100k graph and the 1M city; CCH tests
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r5zc; mkdir -p $O
stop() { rc=$1; [ $rc -eq 124 -o $rc -eq 137 -o $rc -eq 134 -o $rc -eq 139 ] && { echo "GPU step ended rc=$rc: stopping"; exit $rc; }; [ $rc -ne 0 ] && echo "step rc=$rc"; }
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_cch_gpu.py > $O/tests.log 2>&1; stop $?
timeout -k 10 200 python -u bench/cch_customize_bench.py --contexts 6 --check > $O/cust100k_split.jsonl 2>&1; stop $?
ROUTEST_CCH_ARC_HASH=0 timeout -k 10 200 python -u bench/cch_customize_bench.py --contexts 6 > $O/cust100k_b.jsonl 2>&1; stop $?
timeout -k 10 240 python -u bench/cch_customize_bench.py --nodes 1000000 --contexts 3 > $O/cust1m_split.jsonl 2>&1; stop $?
echo done
