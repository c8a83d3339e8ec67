#!/bin/bash
# fused-ANI cost at w = 31 and w = 45 (tools/bench_ani_dest.py)
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/aw
mkdir -p $O
cd $R
for wk in "31 21" "45 30"; do
  timeout -k 10 300 python3 tools/bench_ani_dest.py 8 $wk 2>&1 | grep -v amdgpu.ids >> $O/out.txt || exit 1
done
cat $O/out.txt
