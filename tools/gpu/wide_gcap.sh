#!/bin/bash
# 128-bit layout: whole-call time and the placement kernel's time at group caps 2048 / 1536 / 1024
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/wg
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for gc in 2048 1536 1024; do
  SKS_LAYOUT_GROUP_CAP=$gc SKS_BENCH_KERNELS=join timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t_$gc -o run -- python3 $R/tools/bench_pairs.py 1000 6 family 45 > $O/run_$gc.log 2>&1 || exit 1
  f=$(find $O/t_$gc -name '*kernel_stats.csv' | head -1)
  grep -v amdgpu $O/run_$gc.log | tail -1
  python3 - $f $gc <<'PY'
import csv, re, sys
for r in csv.DictReader(open(sys.argv[1])):
    m = re.search(r"(k_\w+)", r["Name"])
    if m and m.group(1).startswith(("k_gl_", "k_join")):
        print(sys.argv[2], m.group(1), round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
done
