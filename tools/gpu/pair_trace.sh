#!/bin/bash
# kernel timeline of one config-4 all-pairs call (counts only, then with the fused ANI)
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/ptrace
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for m in "counts 31" "ani 31" "counts 45"; do
  read -r kind w <<< "$m"
  m=${kind}_$w
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/t_$m -o run -- python3 $R/tools/pair_call_trace.py run 10 $kind $w > $O/run_$m.log 2>&1 || exit 1
  f=$(find $O/t_$m -name '*kernel_trace.csv' | head -1)
  python3 $R/tools/pair_call_trace.py sum $f > $O/timeline_$m.txt
  tail -3 $O/run_$m.log; cat $O/timeline_$m.txt
done
