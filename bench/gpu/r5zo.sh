# round 5: PMC of the two 256 x 256 K loops (gemm256_kernel drain loop vs gemm256p_kernel phase
# pipeline) at the H = 1024 trainer's shape (bench/gemm_probe.py)
ROOT=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
O=$ROOT/gpurun_out/r5zo; mkdir -p $O
G1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
G2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_LDS_IDX_ACTIVE FETCH_SIZE"
for p in 0 1; do
  i=0
  for G in "$G1" "$G2"; do
    i=$((i+1))
    ROUTEST_GEMM_PIPE=$p timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $G -d $O/p${p}_$i -o g --output-format csv -- python3 $ROOT/bench/gemm_probe.py --iters 10 > $O/p${p}_$i.log 2>&1 || { echo "pass p$p g$i failed rc=$?"; tail -5 $O/p${p}_$i.log; exit 1; }
  done
done
echo pmc done
cd $ROOT
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/t1k -o train --output-format csv -- python3 bench/train_bench.py --hidden 1024 --batch 65536 --steps 30 --warmup 5 --modes fused > $O/t1k.log 2>&1 || { echo "train stats failed rc=$?"; exit 1; }
echo stats done
