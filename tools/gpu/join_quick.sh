# join parity subset + config-4 pair timings (family / unrelated) + bench pairs leg
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/jq
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_rccl.py tests/test_scale.py -m gpu -x -q --timeout 300 --timeout-method thread -k "join or layout or rccl or kernel_ctx or config4" > $O/gputest.log 2>&1
echo "checks done"
cd /tmp && export TMPDIR=/tmp
SKS_BENCH_KERNELS=join timeout -k 10 200 python3 $R/tools/bench_pairs.py 1000 5 family > $O/family.txt 2>&1
SKS_BENCH_KERNELS=join timeout -k 10 200 python3 $R/tools/bench_pairs.py 1000 5 indep > $O/indep.txt 2>&1
SKS_BENCH_KERNELS=join timeout -k 10 200 python3 $R/tools/bench_pairs.py 200 5 family > $O/c5.txt 2>&1
SKS_BENCH_KERNELS=join timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/tools/bench_pairs.py 1000 3 family > $O/traced.txt 2>&1
cd $R
timeout -k 10 300 python3 bench.py --no-sweep --no-e2e --no-c3-sharded --no-c2 --no-cpu-baseline > $O/bench.json 2> $O/bench.err
echo "pairs done"
