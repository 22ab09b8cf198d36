# round 6: 4-rank shared-GPU rehearsal of bench.py with the round-end code; multi-GPU test file in
# shared mode
ROOT=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $ROOT
O=$ROOT/gpurun_out/r6ab; mkdir -p $O
stop() { rc=$1; [ $rc -eq 124 -o $rc -eq 137 -o $rc -eq 134 -o $rc -eq 139 ] && { echo "GPU step ended rc=$rc: stopping"; exit $rc; }; [ $rc -ne 0 ] && echo "step rc=$rc"; }
timeout -k 10 400 env ROUTEST_BENCH_SHARE_GPU=1 python bench.py --gpus 4 --steps 10 --warmup 3 --p50 0 > $O/bench_share4.log 2>&1; stop $?
grep '^{' $O/bench_share4.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['n_gpus'], d['value'], d['schema_problems'], d.get('dp_training',{}).get('ms_per_step'), d.get('dp_training_oneshot',{}).get('ms_per_step') if isinstance(d.get('dp_training_oneshot'),dict) else None)"
timeout -k 10 400 env ROUTEST_TEST_SHARE_GPU=1 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_multigpu.py > $O/multigpu_share.log 2>&1; stop $?
tail -1 $O/multigpu_share.log
echo done
