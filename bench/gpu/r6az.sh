#!/bin/bash
# 2-rank shared-GPU rehearsal WITH the serving sections on rank 0 (two route services per GPU on the
# persisted path), then a second default 1-GPU bench line for the range
ROOT=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $ROOT
O=$ROOT/gpurun_out/r6az; mkdir -p $O
timeout -k 10 500 env ROUTEST_BENCH_SHARE_GPU=1 python bench.py --gpus 2 --steps 10 --warmup 3 > $O/bench_share2.log 2>&1 &&
grep -o '"schema_problems": \[[^]]*\]' $O/bench_share2.log &&
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
rc=$?
echo "rc=$rc"
exit $rc
