# A/B of the all-pairs kernels (config 4 family / independent genomes, config 5 size) + kernel trace
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
timeout -k 10 200 python3 $R/tools/bench_pairs.py 1000 5 family > $R/gpurun_out/pairs_family.txt 2>&1
timeout -k 10 200 python3 $R/tools/bench_pairs.py 1000 5 indep > $R/gpurun_out/pairs_indep.txt 2>&1
timeout -k 10 200 python3 $R/tools/bench_pairs.py 200 5 family > $R/gpurun_out/pairs_200.txt 2>&1
SKS_BENCH_KERNELS=join,postings timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pairs_trace -o run -- python3 $R/tools/bench_pairs.py 1000 3 family > $R/gpurun_out/pairs_traced.txt 2>&1
