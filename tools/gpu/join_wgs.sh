#!/bin/bash
# k_join workgroup-count sweep (SKS_JOIN_WGS) on config 4, then the join tests
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/jw
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_join_dedup.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "carry" > $O/carry.log 2>&1 || { tail -30 $O/carry.log; exit 1; }
tail -1 $O/carry.log
for pass in 1 2; do
  for wgs in 0 "$@"; do
    for m in "family 31" "indep 31" "family 45"; do
      read -r mode w <<< "$m"
      if [ $wgs = 0 ]; then E=""; else E="SKS_JOIN_WGS=$wgs"; fi
      env $E SKS_BENCH_KERNELS=join timeout -k 10 200 python3 tools/bench_pairs.py 1000 6 $mode $w 2>&1 \
        | grep -v amdgpu.ids | sed "s/^/wgs$wgs w$w /" >> $O/ab.txt || exit 1
    done
  done
done
cat $O/ab.txt
