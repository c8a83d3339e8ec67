# whole all-pairs call timings (config 4 family / unrelated, config-5 size) per variant, then kernel times
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/var
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for tag in "$@"; do
  if [ "$tag" = base ]; then L=$R/spaced-kmer-sketching_amd/lib/libsks.so; else L=$R/variants/libsks_$tag.so; fi
  for a in "1000 7 family" "1000 7 indep" "200 7 family"; do
    SKS_LIB=$L SKS_BENCH_KERNELS=join timeout -k 10 200 python3 $R/tools/bench_pairs.py $a 2>&1 | grep -v amdgpu | sed "s/^/$tag /" >> $O/times.txt || exit 1
  done
done
bash $R/tools/gpu/place_variants.sh "$@"
