# A/B of library variants on the config-4 pair call: bash tools/gpu/ab_variants.sh <tag> [<tag> ...]
# ("base" = the tree's libsks.so); family / unrelated genomes and config-5 size, whole call medians
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/abv
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for pass in 1 2; do
  for tag in "$@"; do
    if [ "$tag" = base ]; then L=$R/spaced-kmer-sketching_amd/lib/libsks.so; else L=$R/variants/libsks_$tag.so; fi
    for m in family indep; do
      SKS_LIB=$L SKS_BENCH_KERNELS=join timeout -k 10 120 python3 $R/tools/bench_pairs.py 1000 7 $m 2>&1 | grep -v amdgpu | sed "s/^/$tag p$pass /" >> $O/ab.txt || exit 1
    done
    SKS_LIB=$L SKS_BENCH_KERNELS=join timeout -k 10 120 python3 $R/tools/bench_pairs.py 200 7 family 2>&1 | grep -v amdgpu | sed "s/^/$tag p$pass c5 /" >> $O/ab.txt || exit 1
  done
done
echo done
