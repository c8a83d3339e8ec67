# whole-call times (auto region size, rg1, and variants given), then a pairs-only bench line
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/tb
rm -rf $O; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for tag in auto rg1 "$@"; do
  for a in "1000 7 family" "1000 7 indep" "200 7 family"; do
    case $tag in auto) E="SKS_BENCH_KERNELS=join";; rg1) E="SKS_LAYOUT_RG=1";; *) E="SKS_LIB=$R/variants/libsks_$tag.so";; esac
    env $E SKS_BENCH_KERNELS=join timeout -k 10 200 python3 $R/tools/bench_pairs.py $a 2>&1 | grep -v amdgpu | sed "s/^/$tag /" >> $O/times.txt
  done
done
cd $R
timeout -k 10 400 python3 bench.py --no-e2e --no-c3-sharded --no-c2 --no-sweep --no-cpu-baseline > $O/bench.json 2> $O/bench.err
echo done
