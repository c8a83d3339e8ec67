cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_scale.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/abscan_tests.log 2>&1 || { tail -30 gpurun_out/abscan_tests.log; exit 1; }
tail -2 gpurun_out/abscan_tests.log
for pass in 1 2; do
 for mode in static dyn; do
  if [ $mode = static ]; then export SKS_SCAN_STATIC=1; else unset SKS_SCAN_STATIC; fi
  echo "== $mode pass $pass"
  timeout -k 10 200 python3 tools/bench_scan.py 3000000000 7 1 2>&1 | grep -v amdgpu
  timeout -k 10 200 python3 tools/bench_scan.py 640000000 9 128 2>&1 | grep -v amdgpu
  timeout -k 10 200 python3 tools/bench_scan.py 5000000000 5 1000 2>&1 | grep -v amdgpu
 done
done
