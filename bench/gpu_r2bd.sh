# mixed-traffic soak of the whole app on the GPU services (60 s, 64 clients)
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r2bd; mkdir -p $O
timeout -k 10 300 python -u tools/app_soak.py --seconds 60 --clients 64 > $O/soak.log 2>&1 || exit 1
echo done
