# longer mixed-traffic app soak (150 s, 128 clients) on the GPU services
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r2bl; mkdir -p $O
timeout -k 10 400 python -u tools/app_soak.py --seconds 150 --clients 128 > $O/soak.log 2>&1 || exit 1
echo done
