#!/bin/bash
# k_join A/B: this tree's library against variants/libsks_<tag>.so on config 4
# (family, unrelated, w = 45), two alternating passes; then the join parity
# tests and the phase stamps of this tree's kernel (variants/libsks_jstamp.so)
#   bash tools/gpu/join_ab.sh prevjoin
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/jab
mkdir -p $O
cd $R
TAGS=("$@")
for pass in 1 2; do
  for lib in base "${TAGS[@]}"; do
    if [ $lib = base ]; then L=$R/spaced-kmer-sketching_amd/lib/libsks.so; else L=$R/variants/libsks_$lib.so; fi
    for m in "family 31" "indep 31" "family 45"; do
      read -r mode w <<< "$m"
      SKS_LIB=$L SKS_BENCH_KERNELS=join timeout -k 10 200 python3 tools/bench_pairs.py 1000 6 $mode $w 2>&1 \
        | grep -v amdgpu.ids | sed "s/^/$lib w$w /" >> $O/ab.txt || exit 1
    done
  done
done
cat $O/ab.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "join or config4 or config5 or intersect or fused_ani or all_vs_all" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
SKS_LIB=$R/variants/libsks_jstamp.so SKS_BENCH_KERNELS=join timeout -k 10 200 python3 tools/bench_pairs.py 1000 2 family 31 2>&1 | grep stamps | tail -1
