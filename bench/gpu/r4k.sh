# round 4: route HTTP serving after the assembly fast paths (reactor / client thread split), soak
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
export TMPDIR=/tmp
O=$ROOT/gpurun_out/r4k; mkdir -p $O
for T in 8 4; do
  for CT in 8 4; do
    timeout -k 10 200 python3 bench/route_http_bench.py --provider graph --modes native --seconds 5 --threads $T --client-threads $CT > $O/http_${T}_${CT}.log 2>&1 || { tail -20 $O/http_${T}_${CT}.log; exit 1; }
    echo "threads=$T client=$CT $(tail -1 $O/http_${T}_${CT}.log | cut -c1-700)"
  done
done
timeout -k 10 300 python3 tools/app_soak.py --stack --clients 128 --seconds 20 > $O/soak.log 2>&1 || { tail -20 $O/soak.log; exit 5; }
tail -1 $O/soak.log | cut -c1-2000
