# config-4 pair timings (family / unrelated / config-5 size) + layout phase stamps + kernel trace
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/ab
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for m in family indep; do
  SKS_BENCH_KERNELS=join timeout -k 10 200 python3 $R/tools/bench_pairs.py 1000 7 $m > $O/$m.txt 2>&1
done
SKS_BENCH_KERNELS=join timeout -k 10 200 python3 $R/tools/bench_pairs.py 200 7 family > $O/c5.txt 2>&1
SKS_LIB=$R/variants/libsks_stamps.so SKS_BENCH_KERNELS=join timeout -k 10 200 python3 $R/tools/bench_pairs.py 1000 2 family > $O/stamps_family.txt 2>&1
SKS_LIB=$R/variants/libsks_stamps.so SKS_BENCH_KERNELS=join timeout -k 10 200 python3 $R/tools/bench_pairs.py 1000 2 indep > $O/stamps_indep.txt 2>&1
for m in family indep; do
  SKS_BENCH_KERNELS=join timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$m -o run -- python3 $R/tools/bench_pairs.py 1000 3 $m > $O/traced_$m.txt 2>&1
done
echo done
