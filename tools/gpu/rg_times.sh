# join / layout tests, then whole-call and kernel times with the layout's region
# size forced (SKS_LAYOUT_RG=1,2,3) and chosen by the build (auto), plus any
# library variants given as arguments
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/rg
rm -rf $O; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_join_dedup.py tests/test_scale.py tests/test_gpu_parity.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -k "join or layout or config4 or intersect or fused" > $O/tests.log 2>&1
echo "tests: $(tail -1 $O/tests.log)"
cd /tmp && export TMPDIR=/tmp
for rg in auto 1 2 3; do
  for a in "1000 7 family" "1000 7 indep" "200 7 family"; do
    if [ $rg = auto ]; then E=; else E="SKS_LAYOUT_RG=$rg"; fi
    env $E SKS_BENCH_KERNELS=join timeout -k 10 200 python3 $R/tools/bench_pairs.py $a 2>&1 | grep -v amdgpu | sed "s/^/rg$rg /" >> $O/times.txt
  done
done
for tag in "$@"; do
  for a in "1000 7 family" "1000 7 indep" "200 7 family"; do
    SKS_LIB=$R/variants/libsks_$tag.so SKS_BENCH_KERNELS=join timeout -k 10 200 python3 $R/tools/bench_pairs.py $a 2>&1 | grep -v amdgpu | sed "s/^/$tag /" >> $O/times.txt
  done
done
echo done
