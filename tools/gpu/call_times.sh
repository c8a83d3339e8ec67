#!/bin/bash
# whole-call times: sks_intersect_sym (ctx events) and sks_all_pairs_ani counts (sync to sync) on
# config 4 family / unrelated and config-5 size, two passes; then the intersect / join tests
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/ct
mkdir -p $O
cd $R
for pass in 1 2; do
  for m in "1000 family 31" "1000 indep 31" "200 family 31" "1000 family 45"; do
    read -r n mode w <<< "$m"
    SKS_BENCH_KERNELS=join,onecall timeout -k 10 200 python3 tools/bench_pairs.py $n 8 $mode $w 2>&1 \
      | grep -v amdgpu.ids | sed "s/^/w$w /" >> $O/ab.txt || exit 1
  done
done
cat $O/ab.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "intersect or join or config or dedup or layout or scale or wide" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
