# round 4: PMC counters of the v3 training kernels that run (train_bwd_kernel, eta_mlp3_train_fwd_kernel,
# wgrad_reduce, adamw) at 64k and 1M rows (H=256), and of the wide trainer's GEMMs (H=1024, 64k rows);
# CCH kernel stats after the sweep/unpack work
ROOT=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
O=$ROOT/gpurun_out/r4i; mkdir -p $O
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/cchprof -o cch --output-format csv -- python3 $ROOT/bench/cch_bench.py --reps 2 > $O/cchprof.log 2>&1 || { tail -20 $O/cchprof.log; exit 1; }
G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_INSTS_VMEM GRBM_GUI_ACTIVE"
G2="SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES"
G3="FETCH_SIZE"
G4="WRITE_SIZE"
i=0
for G in "$G1" "$G2" "$G3" "$G4"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $G -d $O/t64k$i -o train --output-format csv -- python3 $ROOT/bench/train_bench.py --hidden 256 --batch 65536 --steps 6 --warmup 2 --modes fused > $O/t64k$i.log 2>&1 || exit $((10+i))
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $G -d $O/t1m$i -o train --output-format csv -- python3 $ROOT/bench/train_bench.py --hidden 256 --batch 1048576 --steps 4 --warmup 2 --modes fused > $O/t1m$i.log 2>&1 || exit $((20+i))
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $G -d $O/t1k$i -o train --output-format csv -- python3 $ROOT/bench/train_bench.py --hidden 1024 --batch 65536 --steps 4 --warmup 2 --modes fused > $O/t1k$i.log 2>&1 || exit $((30+i))
done
echo done
cd $ROOT
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 7; }
tail -1 $O/bench.log | cut -c1-300
