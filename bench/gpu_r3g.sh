# round 3: PMC passes for gcn_l1_fused_kernel (+ the GCN training kernels) and the A* kernels, and a
# kernel-stats profile of the training step at 1M rows per GPU (H=256) and H=1024
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r3g; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_INSTS_VMEM GRBM_GUI_ACTIVE"
G2="SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES"
G3="FETCH_SIZE"
G4="WRITE_SIZE"
i=0
for G in "$G1" "$G2" "$G3" "$G4"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $G -d $O/gcn$i -o gcn --output-format csv -- python3 $ROOT/bench/gcn_bench.py --mode replicate --steps 5 --warmup 1 > $O/gcn$i.log 2>&1 || exit $((10+i))
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $G -d $O/astar$i -o astar --output-format csv -- python3 $ROOT/bench/astar_probe.py --repeat 1 > $O/astar$i.log 2>&1 || exit $((20+i))
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/train1m -o train --output-format csv -- python3 $ROOT/bench/train_bench.py --hidden 256 --batch 1048576 --steps 10 --warmup 3 --modes fused > $O/train1m.log 2>&1 || exit 31
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/train1k -o train --output-format csv -- python3 $ROOT/bench/train_bench.py --hidden 1024 --batch 262144 --steps 10 --warmup 3 --modes fused > $O/train1k.log 2>&1 || exit 32
tail -2 $O/train1m.log $O/train1k.log
echo done
