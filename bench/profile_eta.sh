#!/bin/bash
# rocprofv3 recipe (run on the GPU box from the repo root):
#   1) kernel trace + stats of the flagship inference step and of a training run
#   2) PMC counters for the fused kernels in their OWN run (no sys/runtime tracing with --pmc)
set -e
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
OUT=${OUT:-gpurun_out/prof}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/bench_trace -o bench --output-format csv -- \
    python3 bench.py --steps 20 --warmup 5 --p50 0
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/train_trace -o train --output-format csv -- \
    python3 bench/train_bench.py --steps 20 --warmup 5 --modes fused
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_BUSY_CYCLES \
    -d $OUT/pmc1 -o pmc1 --output-format csv -- \
    python3 bench/eta_kernel_sweep.py --batches 1048576 --variants 1 --iters 5 --rounds 1
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES \
    -d $OUT/pmc2 -o pmc2 --output-format csv -- \
    python3 bench/eta_kernel_sweep.py --batches 1048576 --variants 1 --iters 5 --rounds 1
