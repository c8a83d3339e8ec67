# round-4 baseline from the round-3 tree: config-4 pair timings (family / unrelated / config-5 size),
# a kernel trace of the family call, and the default bench line
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r04_base
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
SKS_BENCH_KERNELS=join timeout -k 10 200 python3 $R/tools/bench_pairs.py 1000 7 family > $O/family.txt 2>&1
SKS_BENCH_KERNELS=join timeout -k 10 200 python3 $R/tools/bench_pairs.py 1000 7 indep > $O/indep.txt 2>&1
SKS_BENCH_KERNELS=join timeout -k 10 200 python3 $R/tools/bench_pairs.py 200 7 family > $O/c5.txt 2>&1
SKS_BENCH_KERNELS=join timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/tools/bench_pairs.py 1000 3 family > $O/traced.txt 2>&1
cd $R
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err
echo done
