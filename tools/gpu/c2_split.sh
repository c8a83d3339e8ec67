#!/bin/bash
# config-2 single-build split: wall time per build and every kernel's time, for the
# default single-genome post path and the fused one (SKS_FUSED_SINGLE=1)
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/c2
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in default fused; do
  if [ $v = fused ]; then export SKS_FUSED_SINGLE=1; else unset SKS_FUSED_SINGLE; fi
  timeout -k 10 120 python3 $R/tools/bench_c2.py 40 1 > $O/wall_$v.txt 2>&1 || exit 1
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t_$v -o run -- python3 $R/tools/bench_c2.py 40 1 > $O/prof_$v.log 2>&1 || exit 1
  f=$(ls $O/t_$v/*/run_kernel_stats.csv 2>/dev/null | head -1)
  [ -z "$f" ] && f=$(find $O/t_$v -name '*kernel_stats.csv' | head -1)
  cut -c1-200 "$f" > $O/stats_$v.csv
done
cat $O/wall_*.txt
