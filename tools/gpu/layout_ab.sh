# join pair phase after the probe-loop fix: grouped vs hash layout build, family / indep, + kernel trace and bench pairs leg
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/ab
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
SKS_BENCH_KERNELS=join timeout -k 10 200 python3 $R/tools/bench_pairs.py 1000 5 family > $O/grouped_family.txt 2>&1
SKS_BENCH_KERNELS=join SKS_JOIN_HASH_LAYOUT=1 timeout -k 10 200 python3 $R/tools/bench_pairs.py 1000 5 family > $O/hash_family.txt 2>&1
SKS_BENCH_KERNELS=join timeout -k 10 200 python3 $R/tools/bench_pairs.py 1000 5 indep > $O/grouped_indep.txt 2>&1
SKS_BENCH_KERNELS=join SKS_JOIN_HASH_LAYOUT=1 timeout -k 10 200 python3 $R/tools/bench_pairs.py 1000 5 indep > $O/hash_indep.txt 2>&1
SKS_BENCH_KERNELS=join timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/tools/bench_pairs.py 1000 3 family > $O/traced.txt 2>&1
echo "pairs done"
cd $R
timeout -k 10 300 python3 bench.py --no-sweep --no-e2e --no-c3-sharded --no-c2 --no-cpu-baseline > $O/bench.json 2> $O/bench.err
echo "bench done"
