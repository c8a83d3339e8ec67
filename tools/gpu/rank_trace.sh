#!/bin/bash
# kernel timeline of one rank's pair step at N = 8 (tools/rank_sim.py replay)
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/rtrace
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for rk in 0 5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/t_$rk -o run -- python3 $R/tools/rank_sim.py trace 8 $rk > $O/run_$rk.log 2>&1 || exit 1
  f=$(find $O/t_$rk -name '*kernel_trace.csv' | head -1)
  python3 - $f <<'PY' > $O/timeline_$rk.txt
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
# the last call: from the last k_gl_prep that follows a gap of > 50 us (the call's first launch)
starts = [i for i in range(1, len(rows)) if int(rows[i]["Start_Timestamp"]) - int(rows[i - 1]["End_Timestamp"]) > 50000]
last = rows[starts[-1]:]
t0 = int(last[0]["Start_Timestamp"]); pe = t0
for r in last:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(s - t0) / 1e3:8.1f} us dur {(e - s) / 1e3:7.1f} gap {(s - pe) / 1e3:6.1f}  {r['Kernel_Name'].split('(')[0][-50:]}")
    pe = e
print(f"span {(pe - t0) / 1e3:.1f} us")
PY
  grep -v amdgpu $O/run_$rk.log | tail -1; cat $O/timeline_$rk.txt
done
