#!/bin/bash
# Round profile (GPU box, repo root): kernel trace + stats of the default bench
# command, then separate PMC passes (MI355X_MICROARCH.md: FETCH_SIZE and
# WRITE_SIZE cannot share a pass; FETCH_SIZE reads 1/2 of a wide coalesced
# stream on gfx950 and is doubled by tools/traffic_from_pmc.py), then two SQ
# groups for VALU / wait breakdown of the scan kernel.
#   bash tools/profile_round.sh r01
set -e
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/round_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
# --inflight 1: every scan launch runs alone, so the trace average is the
# kernel time bench.py reports for the roofline (its serial pass); the end-to-end
# and one-genome-sharded sections (smaller launches of the same kernel) are off
ARGS="$R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --inflight 1 --no-e2e --no-c3-sharded"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $ARGS > $OUT/bench_traced.json 2> $OUT/trace.log
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 $ARGS --no-pairs --no-sweep > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 $ARGS --no-pairs --no-sweep > $OUT/write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU --output-format csv -d $OUT/sq/p1 -o run -- python3 $ARGS --no-pairs --no-sweep > $OUT/sq1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq/p2 -o run -- python3 $ARGS --no-pairs --no-sweep > $OUT/sq2.log 2>&1
echo profile done
