# two-level join layout: join/layout/RCCL/scale tests, pair timing vs the round-2 hash build, trace, bench pairs
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/lc
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_rccl.py tests/test_scale.py tests/test_facade.py -m gpu -x -q --timeout 200 --timeout-method thread -k "join or rccl or config4 or layout or kernel or many_sketches or intersect or pairwise" > $O/gputest.log 2>&1
echo "gpu tests done"
cd /tmp && export TMPDIR=/tmp
SKS_BENCH_KERNELS=join timeout -k 10 200 python3 $R/tools/bench_pairs.py 1000 5 family > $O/grouped_family.txt 2>&1
SKS_JOIN_HASH_LAYOUT=1 SKS_BENCH_KERNELS=join timeout -k 10 200 python3 $R/tools/bench_pairs.py 1000 5 family > $O/hash_family.txt 2>&1
SKS_BENCH_KERNELS=join timeout -k 10 200 python3 $R/tools/bench_pairs.py 1000 5 indep > $O/grouped_indep.txt 2>&1
SKS_BENCH_KERNELS=join timeout -k 10 200 python3 $R/tools/bench_pairs.py 200 5 family > $O/grouped_200.txt 2>&1
SKS_BENCH_KERNELS=join timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/tools/bench_pairs.py 1000 3 family > $O/traced.txt 2>&1
cd $R
timeout -k 10 300 python3 bench.py --no-sweep --no-e2e --no-c3-sharded --no-c2 --no-cpu-baseline > $O/bench.json 2> $O/bench.err
echo "pairs done"
