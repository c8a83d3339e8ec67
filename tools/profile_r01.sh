#!/bin/bash
# Profiling recipe (run on the GPU box via gpurun from the repo root):
#   kernel trace + stats, then separate PMC passes (MI355X_MICROARCH.md rocprofv3 notes:
#   FETCH_SIZE and WRITE_SIZE cannot share a pass; FETCH_SIZE reads 1/2 of a wide
#   coalesced stream on gfx950, so it is doubled before use).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
ARGS="$R/bench.py --steps 3 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $ARGS > $OUT/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 $ARGS --no-pairs > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 $ARGS --no-pairs > $OUT/write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU --output-format csv -d $OUT/valu -o run -- python3 $ARGS --no-pairs > $OUT/valu.log 2>&1
echo profile done
