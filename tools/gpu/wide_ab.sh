#!/bin/bash
# 128-bit layout A/B: this tree against variants/libsks_<tag>.so, the config-4 w = 45 call
# (two alternating passes) and the placement kernel's mean time; then the 128-bit tests
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/wab
mkdir -p $O
cd $R
for pass in 1 2; do
  for lib in base "$@"; do
    if [ $lib = base ]; then L=$R/spaced-kmer-sketching_amd/lib/libsks.so; else L=$R/variants/libsks_$lib.so; fi
    for m in "family 45" "indep 45"; do
      read -r mode w <<< "$m"
      SKS_LIB=$L SKS_BENCH_KERNELS=join timeout -k 10 200 python3 tools/bench_pairs.py 1000 6 $mode $w 2>&1 \
        | grep -v amdgpu.ids | sed "s/^/$lib w$w /" >> $O/ab.txt || exit 1
    done
  done
done
cat $O/ab.txt
cd /tmp && export TMPDIR=/tmp
for lib in base "$@"; do
  if [ $lib = base ]; then L=$R/spaced-kmer-sketching_amd/lib/libsks.so; else L=$R/variants/libsks_$lib.so; fi
  SKS_LIB=$L SKS_BENCH_KERNELS=join timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t_$lib -o run -- python3 $R/tools/bench_pairs.py 1000 4 family 45 > /dev/null 2>&1 || exit 1
  f=$(find $O/t_$lib -name '*kernel_stats.csv' | head -1)
  python3 - $f $lib <<'PY'
import csv, re, sys
for r in csv.DictReader(open(sys.argv[1])):
    m = re.search(r"(k_\w+)", r["Name"])
    if m and m.group(1).startswith(("k_gl_", "k_join")):
        print(sys.argv[2], m.group(1), round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
done
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "wide or dedup or layout or w45 or scale" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
