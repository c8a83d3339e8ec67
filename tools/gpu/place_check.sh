# k_gl_place rewrite: layout contents/buckets, join parity subset, timings + trace
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/pl
mkdir -p $O
cd $R
LV_JOINS=1 timeout -k 10 300 python3 tools/layout_verify.py family 1 > $O/verify_family.txt 2>&1
LV_JOINS=1 timeout -k 10 300 python3 tools/layout_verify.py indep 1 > $O/verify_indep.txt 2>&1
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_rccl.py -m gpu -x -q --timeout 300 --timeout-method thread -k "join or layout or rccl" > $O/gputest.log 2>&1
echo "checks done"
cd /tmp && export TMPDIR=/tmp
SKS_BENCH_KERNELS=join timeout -k 10 200 python3 $R/tools/bench_pairs.py 1000 5 family > $O/family.txt 2>&1
SKS_BENCH_KERNELS=join timeout -k 10 200 python3 $R/tools/bench_pairs.py 1000 5 indep > $O/indep.txt 2>&1
SKS_BENCH_KERNELS=join timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/tools/bench_pairs.py 1000 3 family > $O/traced.txt 2>&1
echo "pairs done"
