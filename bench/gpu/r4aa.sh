# round 4: PMC of the training kernels after the register-native slab change (64k rows, H=256)
ROOT=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
O=$ROOT/gpurun_out/r4aa; mkdir -p $O
G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_INSTS_VMEM GRBM_GUI_ACTIVE"
G2="SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
G3="FETCH_SIZE"
G4="WRITE_SIZE"
i=0
for G in "$G1" "$G2" "$G3" "$G4"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $G -d $O/t64k$i -o train --output-format csv -- python3 $ROOT/bench/train_bench.py --hidden 256 --batch 65536 --steps 6 --warmup 2 --modes fused > $O/t64k$i.log 2>&1 || exit $((10+i))
done
echo done
