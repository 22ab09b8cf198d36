# round 4: native route tests (hop edges from the GPU), route HTTP, training PMC (v3 kernels), bench.py
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
export TMPDIR=/tmp
O=$ROOT/gpurun_out/r4m; mkdir -p $O
nproc > $O/cpus.txt; cat /sys/fs/cgroup/cpu.max >> $O/cpus.txt 2>/dev/null || true
timeout -k 10 250 python -u -m pytest tests/test_frontend_gpu.py -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 2; }
tail -1 $O/pytest.log
timeout -k 10 200 python3 bench/route_http_bench.py --provider graph --modes native --seconds 6 --threads 8 --client-threads 8 > $O/http.log 2>&1 || { tail -20 $O/http.log; exit 3; }
tail -1 $O/http.log | cut -c1-700
bash bench/gpu/r4i.sh
