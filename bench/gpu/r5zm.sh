# round 5: mixed-traffic soak of the serving stack with the round-end code (predict, batched
# predict, routes persisted with ML ETA, history reads / deletes, health, metrics over real sockets)
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r5zm; mkdir -p $O
stop() { rc=$1; [ $rc -eq 124 -o $rc -eq 137 -o $rc -eq 134 -o $rc -eq 139 ] && { echo "GPU step ended rc=$rc: stopping"; exit $rc; }; [ $rc -ne 0 ] && echo "step rc=$rc"; }
timeout -k 10 240 python3 -u tools/app_soak.py --stack --clients 256 --seconds 60 > $O/soak.log 2>&1; stop $?
tail -1 $O/soak.log | cut -c1-2500
