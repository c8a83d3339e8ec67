#!/bin/bash
# the multi-rank rehearsals (gloo 2/3 ranks on GPU 0, RCCL world 1: native and exchange path),
# then the 128-bit layout A/B (this tree against variants/libsks_nostage.so) and its tests
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
timeout -k 10 1000 bash tools/gpu/rehearse_ranks.sh || exit 1
for f in gpurun_out/reh/*.json; do
  echo "$f"; python3 -c "
import json,sys
l=[x for x in open('$f') if x.startswith('{')]
d=json.loads(l[-1]) if l else {}
p=d.get('pairs',{})
print(' pairs ms', p.get('ms_pair_phase'), 'counts', p.get('ms_counts_phase'), 'ani_mean', p.get('ani_mean_all_pairs'))
pw=d.get('pairs_wide',{})
print(' wide ms', pw.get('ms_pair_phase'), 'ani_mean', pw.get('ani_mean_all_pairs'))"
done
O=$R/gpurun_out/wab
mkdir -p $O
for pass in 1 2; do
  for lib in base nostage; do
    if [ $lib = base ]; then L=$R/spaced-kmer-sketching_amd/lib/libsks.so; else L=$R/variants/libsks_$lib.so; fi
    SKS_LIB=$L SKS_BENCH_KERNELS=join timeout -k 10 200 python3 tools/bench_pairs.py 1000 6 family 45 2>&1 \
      | grep -v amdgpu.ids | sed "s/^/$lib /" >> $O/ab.txt || exit 1
  done
done
cat $O/ab.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "wide" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
