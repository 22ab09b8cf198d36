# A* two-stage sweep: lane-kernel pop budget x wave-stage band width (run on the GPU box)
cd $GRAFT_REPO_ROOT
O=gpurun_out/asweep; mkdir -p $O
for cfg in ${SWEEP:-3000:10 3000:5 2000:10 4000:10 3000:2}; do
  set -- ${cfg/:/ }
  ROUTEST_ASTAR_LANE_POPS=$1 ROUTEST_ASTAR_DELTA=$2 timeout -k 10 150 python -u bench/astar_tail.py > $O/t_$1_$2.log 2>&1 || exit 1
done
echo done
