# elastic restart on the fused HIP trainer (2 ranks on GPU 0) + round-2 PMC passes of the training step
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r2av; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_elastic.py -x -v -m gpu --timeout 280 --timeout-method thread > $O/pytest_elastic.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_INSTS_VMEM GRBM_GUI_ACTIVE"
G2="SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES"
G3="FETCH_SIZE"
G4="WRITE_SIZE"
i=0
for G in "$G1" "$G2" "$G3" "$G4"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $G -d $O/pmc$i -o train --output-format csv -- python3 $ROOT/bench/train_bench.py --hidden 256 --batch 65536 --steps 5 --warmup 2 --modes fused > $O/pmc$i.log 2>&1 || exit $((10+i))
done
echo done
