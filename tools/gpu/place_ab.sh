# join/layout parity subset, then config-4 pair timings (family / unrelated / config-5 size) and a kernel trace
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/pl
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_join_dedup.py tests/test_gpu_parity.py tests/test_scale.py tests/test_rccl.py -m gpu -x -q --timeout 200 --timeout-method thread -k "dedup or join or layout or intersect or wide or sketches_tiled or adversarial or config4 or all_vs_all" > $O/tests.log 2>&1
echo tests ok
cd /tmp && export TMPDIR=/tmp
for m in family indep; do
  SKS_BENCH_KERNELS=join timeout -k 10 200 python3 $R/tools/bench_pairs.py 1000 7 $m > $O/$m.txt 2>&1
done
SKS_BENCH_KERNELS=join timeout -k 10 200 python3 $R/tools/bench_pairs.py 200 7 family > $O/c5.txt 2>&1
for m in family indep; do
SKS_BENCH_KERNELS=join timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$m -o run -- python3 $R/tools/bench_pairs.py 1000 3 $m > $O/traced_$m.txt 2>&1
done
echo done
for m in family indep; do
  SKS_LIB=$R/variants/libsks_stamps.so SKS_BENCH_KERNELS=join timeout -k 10 200 python3 $R/tools/bench_pairs.py 1000 2 $m > $O/stamps_$m.txt 2>&1
done
echo stamps done
