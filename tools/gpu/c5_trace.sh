#!/bin/bash
# kernel trace of the config-5-size all-pairs call (tools/bench_pairs.py 200 family): per-kernel
# averages and the last call's launch timeline
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/c5t
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
SKS_BENCH_KERNELS=join timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t -o run -- python3 $R/tools/bench_pairs.py 200 8 family > $O/run.log 2>&1 || { tail -5 $O/run.log; exit 1; }
f=$(find $O/t -name '*kernel_trace.csv' | head -1)
python3 - $f <<'PY'
import csv, re, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
names = [re.search(r"(k_\w+)", r["Kernel_Name"]).group(1) if re.search(r"(k_\w+)", r["Kernel_Name"]) else r["Kernel_Name"][:30] for r in rows]
# the last 8 launches: one call
last = rows[-8:]
t0 = int(last[0]["Start_Timestamp"])
for r, n in zip(last, names[-8:]):
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    print(f"{n:24s} start {s/1e3:8.1f} us  end {e/1e3:8.1f} us  dur {(e-s)/1e3:7.1f} us")
PY
