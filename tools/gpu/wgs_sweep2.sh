# k_join grid sweep over the deduplicated layout (SKS_JOIN_WGS = total workgroups), config 4 family / unrelated
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/wgs
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for w in 0 2176 3264 6528 8704; do
  for m in family indep; do
    if [ $w = 0 ]; then E=""; else E="SKS_JOIN_WGS=$w"; fi
    env $E SKS_BENCH_KERNELS=join timeout -k 10 120 python3 $R/tools/bench_pairs.py 1000 7 $m 2>&1 | grep -v amdgpu | sed "s/^/wgs=$w /" >> $O/sweep.txt || exit 1
  done
done
echo done
