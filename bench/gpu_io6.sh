cd $GRAFT_REPO_ROOT
O=gpurun_out/io6; mkdir -p $O; rm -f $O/*.log
for io in host hybrid host hybrid device; do
  timeout -k 10 200 python -u bench.py --rec 6 --io $io --p50 0 >> $O/b_$io.log 2>&1 || exit 2
done
echo done
