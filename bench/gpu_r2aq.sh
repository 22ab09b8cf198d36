# multi-GPU test file: skipped on one GPU; its shared-GPU rehearsal (2 ranks on GPU 0) must pass
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
O=gpurun_out/r2aq; mkdir -p $O
timeout -k 10 120 python -u -m pytest tests/test_multigpu.py -v -rs --timeout 100 --timeout-method thread > $O/pytest_skip.log 2>&1 || exit 1
ROUTEST_TEST_SHARE_GPU=1 timeout -k 10 600 python -u -m pytest tests/test_multigpu.py -x -v --timeout 280 --timeout-method thread > $O/pytest_share.log 2>&1 || exit 2
echo done
