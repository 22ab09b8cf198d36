#!/bin/bash
# per-kernel times of the supernodal customization (rocprofv3 kernel trace)
set -o pipefail
O=gpurun_out/r6ae; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench/cch_customize_bench.py --nodes 100000 --contexts 4 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
find $O/prof -name "*kernel_stats.csv" | head -3
