# range join: parity subset + all-pairs A/B (config 4 family / unrelated, config 5 size) + trace
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/rj
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "kernel or many_sketches or intersect or range" > $O/gputest.log 2>&1 && timeout -k 10 300 python -u -m pytest tests/test_rccl.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/rccl.log 2>&1
echo "tests done"
cd /tmp && export TMPDIR=/tmp
SKS_BENCH_KERNELS=join,range timeout -k 10 200 python3 $R/tools/bench_pairs.py 1000 5 family > $O/pairs_family.txt 2>&1
SKS_BENCH_KERNELS=join,range timeout -k 10 200 python3 $R/tools/bench_pairs.py 1000 5 indep > $O/pairs_indep.txt 2>&1
SKS_BENCH_KERNELS=join,range timeout -k 10 200 python3 $R/tools/bench_pairs.py 200 5 family > $O/pairs_200.txt 2>&1
SKS_BENCH_KERNELS=join,range timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/tools/bench_pairs.py 1000 3 family > $O/pairs_traced.txt 2>&1
echo "pairs done"
