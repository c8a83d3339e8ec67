#!/bin/bash
# Round profile (GPU box, repo root): kernel trace + stats of the default bench
# command, then separate FETCH_SIZE / WRITE_SIZE passes (MI355X_MICROARCH.md:
# they cannot share a pass; FETCH_SIZE reads 1/2 of a wide coalesced stream
# on gfx950 and is doubled by tools/traffic_from_pmc.py).
#   bash tools/profile_round.sh r01
set -e
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/round_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
ARGS="$R/bench.py --steps 5 --warmup 2 --no-cpu-baseline"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $ARGS > $OUT/bench_traced.json 2> $OUT/trace.log
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 $ARGS --no-pairs > $OUT/fetch.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 $ARGS --no-pairs > $OUT/write.log 2>&1
echo profile done
