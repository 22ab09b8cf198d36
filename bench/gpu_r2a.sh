# Round 2, first GPU pass: bench launch contract, default headline bench, fwd16 PMC counters.
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=gpurun_out/r2a; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_bench_contract_gpu.py tests/test_eta_kernel_gpu.py -x -v --timeout 150 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 || exit 2
cd /tmp && export TMPDIR=/tmp
G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_VMEM"
G2="SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA"
for g in 1 2; do
  eval C=\$G$g
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C -d $ROOT/$O/pmc_g$g -o g$g --output-format csv -- python3 $ROOT/bench/eta_kernel_sweep.py --batches 8388608 --variants 17 --iters 5 --rounds 1 > $ROOT/$O/pmc_g$g.log 2>&1 || exit 3
done
echo done
