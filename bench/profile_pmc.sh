#!/bin/bash
# rocprofv3 hardware counters (PMC) for the route scorer (GCN K8) and the training kernels (K3):
# each counter group in its OWN run with --kernel-trace only (no sys/runtime tracing with --pmc).
# Run on the GPU box from the repo root; then: python tools/pmc_summary.py gpurun_out/pmc > profiles/pmc_summary.md
set -e
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
OUT=${OUT:-gpurun_out/pmc}
mkdir -p $OUT
G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_BUSY_CYCLES"
G2="SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES"
run() {  # tag counters... -- cmd
  local tag=$1; shift
  local ctr=()
  while [ "$1" != "--" ]; do ctr+=("$1"); shift; done
  shift
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc "${ctr[@]}" -d $OUT/$tag -o $tag --output-format csv -- "$@" \
      > $OUT/$tag.log 2>&1
}
run gcn_g1 $G1 -- python3 bench/gcn_bench.py --steps 3 --warmup 1 --mode replicate
run gcn_g2 $G2 -- python3 bench/gcn_bench.py --steps 3 --warmup 1 --mode replicate
run train_g1 $G1 -- python3 bench/train_bench.py --steps 3 --warmup 1 --modes fused
run train_g2 $G2 -- python3 bench/train_bench.py --steps 3 --warmup 1 --modes fused
run fwd_g2 $G2 -- python3 bench/eta_kernel_sweep.py --batches 1048576 --variants 3 --iters 3 --rounds 1
# memory traffic (derived counters; optional on this stack)
run gcn_mem FETCH_SIZE WRITE_SIZE -- python3 bench/gcn_bench.py --steps 3 --warmup 1 --mode replicate \
    || echo "derived memory counters unavailable" > $OUT/gcn_mem.unavailable
echo pmc done
