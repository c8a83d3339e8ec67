#!/bin/bash
# k_bottom_fused phase stamps (SKS_FUSE_STAMPS variant) for one 5 Mb genome and
# for a 64-genome batch, then the native / python all-pairs A/B
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out
cd $R
SKS_LIB=$R/variants/libsks_fstamp.so SKS_FUSED_SINGLE=1 timeout -k 10 120 python3 tools/bench_c2.py 6 1 > $O/c2_stamps.txt 2>&1 || exit 1
SKS_LIB=$R/variants/libsks_fstamp.so timeout -k 10 120 python3 tools/bench_c2.py 3 64 >> $O/c2_stamps.txt 2>&1 || exit 1
timeout -k 10 300 python3 tools/bench_ani_dest.py 15 > $O/dest3.txt 2>&1
