#!/bin/bash
# k_join phase split (SKS_JOIN_STAMPS variant) on config 4 family / unrelated /
# w = 45, then the interleaved native / python all-pairs A/B
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/js
mkdir -p $O
cd $R
for m in "family 31" "indep 31" "family 45"; do
  set -- $m
  SKS_LIB=$R/variants/libsks_jstamp.so SKS_BENCH_KERNELS=join timeout -k 10 200 python3 tools/bench_pairs.py 1000 2 $1 $2 \
    > $O/stamps_$1_$2.txt 2>&1 || exit 1
  grep -v amdgpu.ids $O/stamps_$1_$2.txt | tail -3
done
timeout -k 10 300 python3 tools/bench_ani_dest.py 20 > $O/dest.txt 2>&1
grep -v amdgpu.ids $O/dest.txt
