# round 4: observed-trip GCN scorer — training length / learning rate sweep (held-out gain vs router)
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
export TMPDIR=/tmp
O=$ROOT/gpurun_out/r4ab; mkdir -p $O
for cfg in "600 5e-3" "1500 5e-3" "3000 5e-3" "1500 1e-2" "3000 2e-3"; do
  set -- $cfg
  timeout -k 10 200 python3 bench/gcn_observed_bench.py --steps $1 --lr $2 > $O/s$1_lr$2.json 2>$O/s$1_lr$2.err || { tail -20 $O/s$1_lr$2.err; exit 2; }
  python3 -c "import json,sys; d=json.loads(open('$O/s$1_lr$2.json').read().strip().splitlines()[-1]); print('$1 $2', d['gain_vs_router_pct'], d['train_s'], d['path_mse_first_last'])"
done
