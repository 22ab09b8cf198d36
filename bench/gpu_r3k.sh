# round 3: PMC passes for the v3 training kernels (train_bwd_kernel, single-pass forward) at 1M rows
ROOT=$GRAFT_REPO_ROOT
O=$ROOT/gpurun_out/${TAG:-r3k}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_INSTS_VMEM GRBM_GUI_ACTIVE SQ_INSTS_SALU"
G2="SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA"
G3="FETCH_SIZE"
G4="WRITE_SIZE SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS"
i=0
for G in "$G1" "$G2" "$G3" "$G4"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $G -d $O/trainpmc$i -o train --output-format csv -- python3 $ROOT/bench/train_bench.py --hidden 256 --batch 1048576 --steps 4 --warmup 2 --modes fused > $O/trainpmc$i.log 2>&1 || exit $((40+i))
done
echo done
