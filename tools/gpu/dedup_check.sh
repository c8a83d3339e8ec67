# round 4: deduplicated join layout + join — parity subset, then config-4 timings and a kernel trace
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/dd
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_join_dedup.py tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k "dedup or join or layout or intersect or wide or sketches_tiled or adversarial" > $O/tests1.log 2>&1
echo "tests1 ok"
timeout -k 10 400 python -u -m pytest tests/test_scale.py tests/test_rccl.py -m gpu -x -v --timeout 250 --timeout-method thread > $O/tests2.log 2>&1
echo "tests2 ok"
cd /tmp && export TMPDIR=/tmp
SKS_BENCH_KERNELS=join timeout -k 10 200 python3 $R/tools/bench_pairs.py 1000 7 family > $O/family.txt 2>&1
SKS_BENCH_KERNELS=join timeout -k 10 200 python3 $R/tools/bench_pairs.py 1000 7 indep > $O/indep.txt 2>&1
SKS_BENCH_KERNELS=join timeout -k 10 200 python3 $R/tools/bench_pairs.py 200 7 family > $O/c5.txt 2>&1
SKS_BENCH_KERNELS=join timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/tools/bench_pairs.py 1000 3 family > $O/traced.txt 2>&1
echo done
