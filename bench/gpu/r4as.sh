# round 4: PMC of the wide trainer's gemm256_kernel (H=1024 shape) — where its waves spend their cycles
ROOT=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
O=$ROOT/gpurun_out/r4as; mkdir -p $O
G1="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS"
G2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAVES GRBM_GUI_ACTIVE"
G3="FETCH_SIZE"
i=0
for G in "$G1" "$G2" "$G3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $G -d $O/g$i -o gemm --output-format csv -- python3 $ROOT/bench/gemm_probe.py --iters 10 > $O/g$i.log 2>&1 || exit $((10+i))
done
echo done
