# round-4 status from HEAD: full GPU suite, default bench, pair timings (family / unrelated / config-5 size)
# and a kernel trace of the family all-pairs call
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/st
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gputest.log 2>&1
echo "gpu tests done"
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err
echo "bench done"
cd /tmp && export TMPDIR=/tmp
for m in family indep; do
  SKS_BENCH_KERNELS=join timeout -k 10 200 python3 $R/tools/bench_pairs.py 1000 7 $m > $O/$m.txt 2>&1
done
SKS_BENCH_KERNELS=join timeout -k 10 200 python3 $R/tools/bench_pairs.py 200 7 family > $O/c5.txt 2>&1
SKS_BENCH_KERNELS=join timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/tools/bench_pairs.py 1000 3 family > $O/traced.txt 2>&1
echo done
