# round 3: training (h1 recompute A/B + kernel stats at 1M rows, H=1024 stats), GCN training bench,
# PMC passes for gcn_l1_fused_kernel and the A* kernels
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r3g; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_train_gpu.py -x -q --timeout 240 --timeout-method thread > $O/pytest_train.log 2>&1 || { tail -40 $O/pytest_train.log; exit 1; }
tail -2 $O/pytest_train.log
for B in 65536 1048576; do
  for F in 0 1 0 1; do
    ROUTEST_TRAIN_H1_RECOMPUTE=$F timeout -k 10 120 python -u bench/train_bench.py --hidden 256 --batch $B --steps 30 --warmup 5 --modes fused > $O/tb_${B}_$F.log 2>&1 || { tail -20 $O/tb_${B}_$F.log; exit 2; }
    echo "B=$B h1_recompute=$F $(tail -1 $O/tb_${B}_$F.log)" | tee -a $O/train_ab.jsonl
  done
done
timeout -k 10 400 python -u bench/gcn_train_bench.py > $O/gcn_train.log 2>&1 || { tail -30 $O/gcn_train.log; exit 3; }
tail -1 $O/gcn_train.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/train1m -o train --output-format csv -- python3 $ROOT/bench/train_bench.py --hidden 256 --batch 1048576 --steps 10 --warmup 3 --modes fused > $O/train1m.log 2>&1 || exit 31
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/train64k -o train --output-format csv -- python3 $ROOT/bench/train_bench.py --hidden 256 --batch 65536 --steps 20 --warmup 3 --modes fused > $O/train64k.log 2>&1 || exit 32
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/train1k -o train --output-format csv -- python3 $ROOT/bench/train_bench.py --hidden 1024 --batch 65536 --steps 10 --warmup 3 --modes fused > $O/train1k.log 2>&1 || exit 33
G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_INSTS_VMEM GRBM_GUI_ACTIVE"
G2="SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES"
G3="FETCH_SIZE"
G4="WRITE_SIZE"
i=0
for G in "$G1" "$G2" "$G3" "$G4"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $G -d $O/gcn$i -o gcn --output-format csv -- python3 $ROOT/bench/gcn_bench.py --mode replicate --steps 5 --warmup 1 > $O/gcn$i.log 2>&1 || exit $((10+i))
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $G -d $O/astar$i -o astar --output-format csv -- python3 $ROOT/bench/astar_probe.py --repeat 1 > $O/astar$i.log 2>&1 || exit $((20+i))
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $G -d $O/trainpmc$i -o train --output-format csv -- python3 $ROOT/bench/train_bench.py --hidden 256 --batch 1048576 --steps 4 --warmup 2 --modes fused > $O/trainpmc$i.log 2>&1 || exit $((40+i))
done
echo done
