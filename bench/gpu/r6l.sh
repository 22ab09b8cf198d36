# round 6: the work-queue persistent probe with wave-uniform loop exits (acquire vs relaxed polls)
ROOT=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $ROOT
O=$ROOT/gpurun_out/r6l; mkdir -p $O
timeout -k 10 60 tools/probes/bin/kernel_chain_probe 200 > $O/kernel_chain_probe.jsonl 2>&1; rc=$?
cat $O/kernel_chain_probe.jsonl; echo "rc=$rc"
