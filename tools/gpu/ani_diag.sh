#!/bin/bash
# fused-ANI cost split (this tree against diagnostics builds in variants/):
# anidiag1 = the hand-off without the conversion, anidiag2 = no atomic drain
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/anid
mkdir -p $O
cd $R
for pass in 1 2; do
  for lib in base "$@"; do
    if [ $lib = base ]; then L=$R/spaced-kmer-sketching_amd/lib/libsks.so; else L=$R/variants/libsks_$lib.so; fi
    echo "== $lib" >> $O/out.txt
    SKS_LIB=$L timeout -k 10 300 python3 tools/bench_ani_dest.py 8 2>&1 | grep -v amdgpu.ids >> $O/out.txt || exit 1
  done
done
cat $O/out.txt
