# round 6: dW1 epilogue with the relu bit mask (H = 1024): tests + A/B + kernel stats; the bounded
# work-queue probe (acquire poll vs relaxed poll + fence)
ROOT=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $ROOT
O=$ROOT/gpurun_out/r6k; mkdir -p $O
stop() { rc=$1; [ $rc -eq 124 -o $rc -eq 137 -o $rc -eq 134 -o $rc -eq 139 ] && { echo "GPU step ended rc=$rc: stopping"; exit $rc; }; [ $rc -ne 0 ] && echo "step rc=$rc"; }
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_train_gpu.py -k "dw1 or wide" > $O/train_tests.log 2>&1; stop $?
tail -1 $O/train_tests.log; grep -E "FAIL|Error" $O/train_tests.log | head -20
for v in 1 0 1 0; do
  ROUTEST_DW1_EPILOGUE=$v timeout -k 10 180 python -u bench/train_bench.py --hidden 1024 --batch 65536 --steps 50 --warmup 10 --modes fused,graph > $O/train1024_e$v.json 2>$O/train1024_e$v.err; stop $?
  echo "dw1_epilogue=$v $(tail -1 $O/train1024_e$v.json | cut -c120-400)"
done
timeout -k 10 120 python -u bench/train_bench.py --hidden 1024 --batch 262144 --steps 20 --warmup 5 --modes fused > $O/train1024_262k.json 2>$O/train1024_262k.err; stop $?
echo "262k $(tail -1 $O/train1024_262k.json | cut -c120-400)"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/ks1024 -o k --output-format csv -- python3 $ROOT/bench/train_bench.py --hidden 1024 --batch 65536 --steps 30 --warmup 5 --modes fused > $O/ks1024.log 2>&1; echo "ks1024 rc=$?"
timeout -k 10 90 tools/probes/bin/kernel_chain_probe 200 > $O/kernel_chain_probe.jsonl 2>&1; stop $?
cat $O/kernel_chain_probe.jsonl
echo done
