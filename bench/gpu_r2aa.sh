# LDS bank-conflict probe of the training kernel's two W2 read patterns
ROOT=$GRAFT_REPO_ROOT
O=$ROOT/gpurun_out/r2aa; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES -d $O/pmc -o p --output-format csv -- $ROOT/build/lds_probe > $O/probe.log 2>&1 || exit 1
echo done
