# round 5: hardware counters of the CCH QUERY kernels (sweep / meet / unpack / matrix helpers) on
# the 80k-leg batch of bench/cch_bench.py (verdict r4 item 3 asks for sweep_kernel PMC too)
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r5zl; mkdir -p $O
stop() { rc=$1; [ $rc -eq 124 -o $rc -eq 137 -o $rc -eq 134 -o $rc -eq 139 ] && { echo "GPU step ended rc=$rc: stopping"; exit $rc; }; [ $rc -ne 0 ] && echo "step rc=$rc"; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 170 rocprofv3 --kernel-trace --stats -d $O/stats -o q --output-format csv -- python3 $ROOT/bench/cch_bench.py --reps 2 > $O/stats.log 2>&1; stop $?
G1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_VALU SQ_INSTS_SALU"
G2="FETCH_SIZE"
G3="WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"
G4="SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM"
i=0
for G in "$G1" "$G2" "$G3" "$G4"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $G -d $O/pmc$i -o q --output-format csv -- python3 $ROOT/bench/cch_bench.py --reps 1 > $O/pmc$i.log 2>&1; stop $?
done
echo done
