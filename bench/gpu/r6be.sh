#!/bin/bash
# final tree: 4-rank shared-GPU rehearsal (every section, rank 0 serving), then one more 1-GPU line
ROOT=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $ROOT
O=$ROOT/gpurun_out/r6be; mkdir -p $O
timeout -k 10 600 env ROUTEST_BENCH_SHARE_GPU=1 python bench.py --gpus 4 --steps 10 --warmup 3 > $O/bench_share4.log 2>&1 &&
grep -o '"schema_problems": \[[^]]*\]' $O/bench_share4.log &&
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
rc=$?; echo "rc=$rc"; exit $rc
