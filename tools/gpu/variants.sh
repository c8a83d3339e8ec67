# per library variant (variants/libsks_<tag>.so; "base" = the in-tree build): the
# join / layout parity tests, then the whole all-pairs call times (family / unrelated
# config 4, config-5 size) and the layout / join kernel times (kernel trace)
#   bash tools/gpu/variants.sh base rg0 rg1 ...
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/var
mkdir -p $O
cd $R
for tag in "$@"; do
  if [ "$tag" = base ]; then L=$R/spaced-kmer-sketching_amd/lib/libsks.so; else L=$R/variants/libsks_$tag.so; fi
  SKS_LIB=$L timeout -k 10 400 python -u -m pytest tests/test_join_dedup.py tests/test_scale.py -m gpu -x -q \
    --timeout 300 --timeout-method thread -k "not config5" > $O/tests_$tag.log 2>&1
  echo "$tag tests: $(tail -1 $O/tests_$tag.log)"
done
bash $R/tools/gpu/pairs_times.sh "$@"
echo done
