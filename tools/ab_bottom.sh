#!/bin/bash
# k_bottom_fused A/B over library variants (variants/libsks_<tag>.so, "base" =
# in-tree) on config 4's sketch (1000 x 5 Mb, bottom-s 10000): kernel trace of
# tools/bench_scan.py's 1000-genome build.  GPU box:  bash tools/ab_bottom.sh tag ...
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/ab_bottom
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for tag in base "$@"; do
  lib=$R/variants/libsks_$tag.so
  [ "$tag" = base ] && lib=$R/spaced-kmer-sketching_amd/lib/libsks.so
  echo "== $tag" >> $OUT/ab.log
  SKS_LIB=$lib timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$tag -o run -- python3 $R/tools/bench_scan.py 5000000000 3 1000 >> $OUT/ab.log 2>&1
  grep -h "k_bottom_fused" $OUT/$tag/*kernel_stats.csv | awk -F'",' '{print $2}' >> $OUT/ab.log || true
done
echo done
