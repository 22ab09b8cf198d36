# PMC of the H=256 training step kernels (forward kernel focus): issue mix, waits, busy
ROOT=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
O=$ROOT/gpurun_out/r2s; mkdir -p $O
G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_VMEM"
G2="SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA"
G3="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD"
for g in 1 2 3; do
  eval C=\$G$g
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C -d $O/pmc_g$g -o g$g --output-format csv -- python3 $ROOT/bench/train_bench.py --steps 5 --warmup 2 --modes fused > $O/pmc_g$g.log 2>&1 || exit $g
done
echo done
