# range join quick loop: range-kernel parity subset + all-pairs timing (config 4 family / unrelated)
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/rjq
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "range or kernel_ctx or many_sketches" > $O/gputest.log 2>&1
echo "tests done"
cd /tmp && export TMPDIR=/tmp
SKS_BENCH_KERNELS=join,range timeout -k 10 200 python3 $R/tools/bench_pairs.py 1000 5 family > $O/pairs_family.txt 2>&1
SKS_BENCH_KERNELS=join,range timeout -k 10 200 python3 $R/tools/bench_pairs.py 1000 5 indep > $O/pairs_indep.txt 2>&1
SKS_BENCH_KERNELS=join,range timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/tools/bench_pairs.py 1000 3 family > $O/pairs_traced.txt 2>&1
echo "pairs done"
