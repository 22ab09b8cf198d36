# headline pipeline timeline: kernel + memory-copy trace of bench.py (no counters)
ROOT=$GRAFT_REPO_ROOT
O=$ROOT/gpurun_out/trace; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/t -o hl -- python3 $ROOT/bench.py --steps 30 --warmup 5 --p50 0 --rec16-steps 0 > $O/bench.log 2>&1 || exit 1
echo done
