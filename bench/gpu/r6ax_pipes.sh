#!/bin/bash
# A/B: native route services per GPU (ROUTEST_ROUTE_PIPELINES 1 / 2 / 3) on the same box
ROOT=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $ROOT
O=$ROOT/gpurun_out/r6ax; mkdir -p $O
for k in 2 1 3; do
  ROUTEST_ROUTE_PIPELINES=$k timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_p$k.json 2> $O/bench_p$k.err || exit $?
  echo "pipes $k done"
done
