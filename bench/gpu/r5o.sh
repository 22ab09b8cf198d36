# round 5: what delays cached-context requests while a 1M-city context builds (build-stage timings;
# one builder vs three; builder on all CUs vs a quarter); kernel table of the 64k training step
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r5o; mkdir -p $O
stop() { rc=$1; [ $rc -eq 124 -o $rc -eq 137 -o $rc -eq 134 -o $rc -eq 139 ] && { echo "GPU step ended rc=$rc: stopping"; exit $rc; }; [ $rc -ne 0 ] && echo "step rc=$rc"; }
timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_cch_async_gpu.py tests/test_cch_gpu.py > $O/tests.log 2>&1; stop $?
timeout -k 10 240 python -u bench/route_context_bench.py --nodes 1000000 --concurrency 256 --phases fresh > $O/fresh_default.jsonl 2>$O/fresh_default.err; stop $?
ROUTEST_CCH_BUILDERS=1 timeout -k 10 240 python -u bench/route_context_bench.py --nodes 1000000 --concurrency 256 --phases fresh > $O/fresh_b1.jsonl 2>$O/fresh_b1.err; stop $?
ROUTEST_CCH_BUILDER_CU_SHARE=1 timeout -k 10 240 python -u bench/route_context_bench.py --nodes 1000000 --concurrency 256 --phases fresh > $O/fresh_allcu.jsonl 2>$O/fresh_allcu.err; stop $?
cd /tmp && export TMPDIR=/tmp && cd $ROOT
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/trainprof -o train -- python3 bench/train_bench.py --modes fused --steps 100 --warmup 10 > $O/train_prof.log 2>&1; stop $?
echo done
