# round 6: serving soaks with the round-end code (native front end mixed traffic over sockets; the
# FastAPI app in-process)
ROOT=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $ROOT
O=$ROOT/gpurun_out/r6y; mkdir -p $O
stop() { rc=$1; [ $rc -eq 124 -o $rc -eq 137 -o $rc -eq 134 -o $rc -eq 139 ] && { echo "GPU step ended rc=$rc: stopping"; exit $rc; }; [ $rc -ne 0 ] && echo "step rc=$rc"; }
timeout -k 10 300 python -u tools/app_soak.py --stack --seconds 60 --clients 256 > $O/soak_stack.log 2>&1; stop $?
tail -3 $O/soak_stack.log | cut -c1-600
timeout -k 10 240 python -u tools/app_soak.py --seconds 30 --clients 64 > $O/soak_app.log 2>&1; stop $?
tail -3 $O/soak_app.log | cut -c1-600
echo done
