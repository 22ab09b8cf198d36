#!/bin/bash
# per-service chunk cap (16 / k chunks per parallel_chunks call): two services everywhere vs auto
ROOT=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $ROOT
O=$ROOT/gpurun_out/r6bb; mkdir -p $O
ROUTEST_ROUTE_PIPELINES=2 timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_p2cap.json 2> $O/p2cap.err &&
echo p2cap &&
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_auto.json 2> $O/auto.err
rc=$?; echo "rc=$rc"; exit $rc
