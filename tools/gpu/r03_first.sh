# Round 3 first GPU pass: GPU tests, default bench, all-pairs kernel A/B.
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r03a
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gputest.log 2>&1
echo "gpu tests done"
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err
echo "bench done"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 python3 $R/tools/bench_pairs.py 1000 5 family > $O/pairs_family.txt 2>&1
timeout -k 10 200 python3 $R/tools/bench_pairs.py 1000 5 indep > $O/pairs_indep.txt 2>&1
timeout -k 10 200 python3 $R/tools/bench_pairs.py 200 5 family > $O/pairs_200.txt 2>&1
SKS_BENCH_KERNELS=join,postings timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pairs_trace -o run -- python3 $R/tools/bench_pairs.py 1000 3 family > $O/pairs_traced.txt 2>&1
echo "pairs done"
