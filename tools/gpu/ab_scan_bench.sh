#!/bin/bash
# config-3 bench line (HBM-resident 3 Gb genome, 3 builds in flight) with the
# scan's static tile ranges (SKS_SCAN_STATIC=1) against the dynamic tile queue,
# alternating, two passes; prints value / ms_per_step / scan kernel mean
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
C3="--no-pairs --no-sweep --no-e2e --no-c3-sharded --no-c2 --no-cpu-baseline --steps 20 --warmup 2"
for pass in 1 2; do
  for mode in static dyn; do
    if [ $mode = static ]; then export SKS_SCAN_STATIC=1; else unset SKS_SCAN_STATIC; fi
    timeout -k 10 300 python3 bench.py $C3 > /tmp/ab_$mode.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.loads(open('/tmp/ab_$mode.json').read().strip().splitlines()[-1]); print('$mode p$pass', round(d['value']/1e9,1), 'Gk/s', round(d['ms_per_step'],3), 'ms/step scan', round(d['roofline']['kernel_ms'],3), round(d['roofline']['kernel_ms_median'],3))"
  done
done
