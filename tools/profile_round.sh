#!/bin/bash
# Round profile (GPU box, repo root):  bash tools/profile_round.sh r02
# 1. kernel trace + stats of the DEFAULT bench command (bench.py --steps 20
#    --warmup 2, what the driver runs); the scan launches bench.py times are the
#    serial pass, dispatches [warmup, warmup + steps) of the config-3 scan kernel.
# 2. PMC passes over the same command limited to its config-3 part (identical
#    scan dispatch sequence): FETCH_SIZE and WRITE_SIZE in separate passes
#    (MI355X_MICROARCH.md: they cannot share one; FETCH_SIZE reads 1/2 of a wide
#    coalesced stream on gfx950 and is doubled in tools/summarize_round.py), then
#    two SQ groups for the scan kernel.
# 3. SQ groups over tools/bench_pairs.py (config 4): k_join, k_bottom_fused.
# 4. tools/summarize_round.py -> gpurun_out/round_<tag>/summary (copy to profiles/<tag>).
set -e
TAG=$1
STEPS=${STEPS:-20}; WARMUP=${WARMUP:-2}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/round_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
ARGS="$R/bench.py --steps $STEPS --warmup $WARMUP"
C3="--no-pairs --no-sweep --no-e2e --no-c3-sharded --no-c2 --no-cpu-baseline"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $ARGS > $OUT/bench_traced.json 2> $OUT/trace.log
echo "trace done"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 $ARGS $C3 > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 $ARGS $C3 > $OUT/write.log 2>&1
echo "traffic done"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU --output-format csv -d $OUT/sq/p1 -o run -- python3 $ARGS $C3 > $OUT/sq1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq/p2 -o run -- python3 $ARGS $C3 > $OUT/sq2.log 2>&1
echo "scan counters done"
SKS_BENCH_KERNELS=join timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU --output-format csv -d $OUT/pairs/p1 -o run -- python3 $R/tools/bench_pairs.py 1000 2 > $OUT/pairs1.log 2>&1
SKS_BENCH_KERNELS=join timeout -k 10 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE --output-format csv -d $OUT/pairs/p2 -o run -- python3 $R/tools/bench_pairs.py 1000 2 > $OUT/pairs2.log 2>&1
SKS_BENCH_KERNELS=join timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU --output-format csv -d $OUT/pairs_wide/p1 -o run -- python3 $R/tools/bench_pairs.py 1000 2 family 45 > $OUT/pairsw1.log 2>&1
SKS_BENCH_KERNELS=join timeout -k 10 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE --output-format csv -d $OUT/pairs_wide/p2 -o run -- python3 $R/tools/bench_pairs.py 1000 2 family 45 > $OUT/pairsw2.log 2>&1
# k_join's memory side: bytes past L2 (FETCH_SIZE: L2-to-fabric requests, Infinity-Cache hits
# included) and the L2 hit rate, one pass each
SKS_BENCH_KERNELS=join timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pairs_mem/p1 -o run -- python3 $R/tools/bench_pairs.py 1000 2 > $OUT/pairsm1.log 2>&1
SKS_BENCH_KERNELS=join timeout -k 10 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/pairs_mem/p2 -o run -- python3 $R/tools/bench_pairs.py 1000 2 > $OUT/pairsm2.log 2>&1
echo "pair counters done"
python3 $R/tools/summarize_round.py $OUT $OUT/summary $WARMUP $STEPS
echo profile done
