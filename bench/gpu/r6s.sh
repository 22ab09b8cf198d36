# round 6: PMC passes (one counter group per run) over the H = 1024 training step's kernels:
# wgrad256<32,4> (default), gemm256p<1>, gemm256p<3> (dW1 epilogue)
ROOT=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $ROOT
O=$ROOT/gpurun_out/r6s; mkdir -p $O
G1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
G2="FETCH_SIZE TCC_HIT_sum"
G3="WRITE_SIZE TCC_MISS_sum"
G4="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAVE_CYCLES"
i=0
for G in "$G1" "$G2" "$G3" "$G4"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $G -d $O/pmc_$i -o p --output-format csv -- python3 $ROOT/bench/train_bench.py --hidden 1024 --batch 65536 --steps 3 --warmup 1 --modes fused > $O/pmc_$i.log 2>&1; rc=$?
  echo "pass $i rc=$rc"; ls $O/pmc_$i | head -3
  [ $rc -eq 0 ] || [ $rc -eq 139 ] || break
done
echo done
