#!/bin/bash
# kernel-traced config-4 family pair run per library variant; prints the layout kernels
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/ab_layout
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for tag in base "$@"; do
  lib=$R/variants/libsks_$tag.so
  [ "$tag" = base ] && lib=$R/spaced-kmer-sketching_amd/lib/libsks.so
  SKS_LIB=$lib timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$tag -o run -- python3 $R/tools/bench_pairs.py 1000 5 family > $OUT/$tag.log 2>&1
  echo "== $tag"; grep -h "k_hb_\|k_join" $OUT/$tag/*kernel_stats.csv | awk -F, '{split($1,a,"::"); n=a[3]; sub(/\(.*/,"",n); printf "%-14s %8.1f us\n", n, $4/1000}'
done
