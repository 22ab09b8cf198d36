# round 4: MFMA issue-rate probe (tools/probes/mfma_rate_probe.hip), default and -amdgpu-mfma-vgpr-form builds
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=$ROOT/gpurun_out/r4ag; mkdir -p $O
timeout -k 10 60 ./tools/probes/bin/mfma_rate_probe 2000 > $O/probe.jsonl 2>&1 || { cat $O/probe.jsonl; exit 2; }
cat $O/probe.jsonl
true

