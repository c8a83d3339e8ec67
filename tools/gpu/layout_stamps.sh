# k_gl_place phase stamps (SKS_LAYOUT_STAMPS variant) on config 4 family / unrelated and config-5 size
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/stamps
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for m in family indep; do
  SKS_LIB=$R/variants/libsks_lstamp.so SKS_BENCH_KERNELS=join timeout -k 10 200 python3 $R/tools/bench_pairs.py 1000 2 $m > $O/$m.txt 2>&1
done
SKS_LIB=$R/variants/libsks_lstamp.so SKS_BENCH_KERNELS=join timeout -k 10 200 python3 $R/tools/bench_pairs.py 200 2 family > $O/c5.txt 2>&1
echo done
