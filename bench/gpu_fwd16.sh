# 16x16-MFMA forward kernel: numerics tests + device-resident and headline A/B (run on the GPU box)
cd $GRAFT_REPO_ROOT
O=gpurun_out/fwd16; mkdir -p $O; rm -f $O/*.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_eta_kernel_gpu.py -k "forward" > $O/tests.log 2>&1 || exit 1
for v in ${DEV_VARIANTS:-3 17 16 3 17}; do
  timeout -k 10 200 python -u bench.py --io device --variant $v --p50 0 >> $O/dev_$v.log 2>&1 || exit 2
done
for v in ${HYB_VARIANTS:-17 3}; do
  timeout -k 10 200 python -u bench.py --variant $v --p50 0 >> $O/hyb_$v.log 2>&1 || exit 3
done
echo done
