#!/bin/bash
# config-2 build latency, fused vs unfused bottom-s post-processing, 1..64 genomes
set -e
cd ${GRAFT_REPO_ROOT:-$(pwd)}
for k in 1 2 4 8 16 32 64; do
  timeout -k 10 120 python3 tools/bench_c2.py 12 $k
  SKS_NO_FUSED_BOTTOM=1 timeout -k 10 120 python3 tools/bench_c2.py 12 $k
done
