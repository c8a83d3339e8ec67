# two-level join layout: layout/join parity subset + pair timing + trace
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/lq
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_rccl.py -m gpu -x -q --timeout 200 --timeout-method thread -k "join or layout or kernel_ctx or many_sketches or rccl" > $O/gputest.log 2>&1
echo "gpu tests done"
cd /tmp && export TMPDIR=/tmp
SKS_BENCH_KERNELS=join timeout -k 10 200 python3 $R/tools/bench_pairs.py 1000 5 family > $O/family.txt 2>&1
SKS_BENCH_KERNELS=join timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/tools/bench_pairs.py 1000 3 family > $O/traced.txt 2>&1
echo "pairs done"
