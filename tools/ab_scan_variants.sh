#!/bin/bash
# Scan A/B over library variants (variants/libsks_<tag>.so from
# tools/build_variant.sh, "base" = in-tree): config-3 shape (3 Gb, one genome)
# and config-4 shape (5 Gb in 1000 genomes), FracMinHash 1/1000 and bottom-s
# 10000, median scan ms. Two passes in alternating order.
# GPU box, repo root:  bash tools/ab_scan_variants.sh tag1 tag2 ...
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
for pass in 1 2; do
  for tag in base "$@"; do
    lib=$R/variants/libsks_$tag.so
    [ "$tag" = base ] && lib=$R/spaced-kmer-sketching_amd/lib/libsks.so
    SKS_LIB=$lib timeout -k 10 120 python3 $R/tools/bench_scan.py 3000000000 9 1
    SKS_LIB=$lib timeout -k 10 120 python3 $R/tools/bench_scan.py 5000000000 5 1000
  done
done
