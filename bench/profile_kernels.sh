#!/bin/bash
# rocprofv3 kernel-trace + stats for every GPU workload beyond the flagship (run on the GPU box from
# the repo root).  Each profile runs under its own time limit; the script stops at the first failure.
#   training step (fused HIP path incl. custom wgrad), GCN scorer, batched A*, tree ensemble, greedy CVRP
set -e
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
OUT=${OUT:-gpurun_out/prof2}
mkdir -p $OUT
prof() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs rocprofv3 --kernel-trace --stats -d $OUT/$name -o $name --output-format csv -- "$@" \
      > $OUT/$name.log 2>&1
}
prof train 300 python3 bench/train_bench.py --steps 20 --warmup 5 --modes fused
prof gcn 300 python3 bench/gcn_bench.py --steps 20 --warmup 3 --mode replicate
prof route 400 python3 bench/route_bench.py
prof forest 400 python3 bench/forest_bench.py --reps 5
echo profiles done
