#!/bin/bash
# A/B of k_join builds (variants/libsks_<tag>.so from tools/build_variant.sh, plus
# the in-tree library as "base") on config 4 (family / unrelated genomes) and
# config 5's 200 genomes; the family run is kernel-traced (rocprofv3 --stats),
# so k_join's own average duration is in ab_join/<tag>_family/.
# GPU box, repo root:  bash tools/ab_join.sh tag1 tag2 ...   (AB_BASE= to skip base)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/ab_join
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for tag in ${AB_BASE-base} "$@"; do
  lib=$R/variants/libsks_$tag.so
  [ "$tag" = base ] && lib=$R/spaced-kmer-sketching_amd/lib/libsks.so
  echo "== $tag family (traced)" | tee -a $OUT/ab.log
  SKS_LIB=$lib timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${tag}_family -o run -- python3 $R/tools/bench_pairs.py 1000 5 family >> $OUT/ab.log 2>&1
  grep -h "k_join\|k_tiles" $OUT/${tag}_family/*kernel_stats.csv | cut -c1-200 >> $OUT/ab.log || true
  for mode in ${AB_MODES:-indep}; do
    echo "== $tag $mode" | tee -a $OUT/ab.log
    SKS_LIB=$lib timeout -k 10 120 python3 $R/tools/bench_pairs.py 1000 5 $mode >> $OUT/ab.log 2>&1
  done
  echo "== $tag c5" | tee -a $OUT/ab.log
  SKS_LIB=$lib timeout -k 10 120 python3 $R/tools/bench_pairs.py 200 5 family >> $OUT/ab.log 2>&1
done
echo ab done
