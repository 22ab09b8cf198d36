#!/bin/bash
# no-store route path: two route services per GPU with the shared CPU pool at 16 / 8 workers, and one
# service as the same-box baseline
ROOT=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $ROOT
O=$ROOT/gpurun_out/r6ba; mkdir -p $O
ROUTEST_ROUTE_PIPELINES=2 ROUTEST_CPU_POOL=8 timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_p2_pool8.json 2> $O/p2_pool8.err &&
echo p2pool8 &&
ROUTEST_ROUTE_PIPELINES=2 timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_p2.json 2> $O/p2.err &&
echo p2 &&
ROUTEST_ROUTE_PIPELINES=1 timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_p1.json 2> $O/p1.err
rc=$?; echo "rc=$rc"; exit $rc
