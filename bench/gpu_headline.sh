# Headline bench (default hybrid IO) + kernel trace + 2-rank shared-GPU rehearsal (run on the GPU box)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=gpurun_out/headline; mkdir -p $O
timeout -k 10 240 python -u bench.py > $O/bench.log 2>&1 || exit 1
ROUTEST_BENCH_SHARE_GPU=1 timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 3 --p50 0 > $O/bench_2rank_shared.log 2>&1 || exit 2
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $R/$O/trace -o hybrid --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --p50 0 > $R/$O/trace.log 2>&1 || exit 3
echo done
