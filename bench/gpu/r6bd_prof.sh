#!/bin/bash
# kernel statistics of the whole default bench run with the final tree (trace CSV dropped, stats kept)
ROOT=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $ROOT
O=$ROOT/gpurun_out/r6bd; mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
rc=$?
find $O/prof -name "*kernel_trace.csv" -delete
find $O/prof -name "*.csv" | head -20
exit $rc
