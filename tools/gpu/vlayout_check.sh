# k_join over a value-range layout (SKS_JOIN_VALUE_LAYOUT) vs the hash layout: parity subset + timing + trace
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/vl
mkdir -p $O
cd $R
SKS_JOIN_VALUE_LAYOUT=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "kernel_ctx or many_sketches or join or intersect" > $O/gputest.log 2>&1
echo "tests done"
cd /tmp && export TMPDIR=/tmp
SKS_BENCH_KERNELS=join timeout -k 10 200 python3 $R/tools/bench_pairs.py 1000 5 family > $O/hash_family.txt 2>&1
SKS_JOIN_VALUE_LAYOUT=1 SKS_BENCH_KERNELS=join timeout -k 10 200 python3 $R/tools/bench_pairs.py 1000 5 family > $O/value_family.txt 2>&1
SKS_JOIN_VALUE_LAYOUT=1 SKS_BENCH_KERNELS=join timeout -k 10 200 python3 $R/tools/bench_pairs.py 1000 5 indep > $O/value_indep.txt 2>&1
SKS_JOIN_VALUE_LAYOUT=1 SKS_BENCH_KERNELS=join timeout -k 10 200 python3 $R/tools/bench_pairs.py 200 5 family > $O/value_200.txt 2>&1
SKS_JOIN_VALUE_LAYOUT=1 SKS_BENCH_KERNELS=join timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/tools/bench_pairs.py 1000 3 family > $O/traced.txt 2>&1
echo "pairs done"
