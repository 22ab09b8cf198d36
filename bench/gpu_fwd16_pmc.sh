# PMC counters: 32x32 (variant 3) vs 16x16 NH=4 (variant 17) forward kernels, 8M rows, random weights
ROOT=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
OUT=$ROOT/gpurun_out/pmc16; mkdir -p $OUT
G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
G2="SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES"
for v in 3 17; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $G1 -d $OUT/g1_$v -o g1 --output-format csv -- python3 $ROOT/bench/eta_kernel_sweep.py --batches 8388608 --variants $v --iters 5 --rounds 1 > $OUT/g1_$v.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $G2 -d $OUT/g2_$v -o g2 --output-format csv -- python3 $ROOT/bench/eta_kernel_sweep.py --batches 8388608 --variants $v --iters 5 --rounds 1 > $OUT/g2_$v.log 2>&1 || exit 2
done
echo done
