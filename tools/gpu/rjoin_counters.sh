# range join vs hash join: parity subset, timing, and SQ counters per kernel (config 4 family)
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/rjc
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "kernel or many_sketches or intersect or range" > $O/gputest.log 2>&1
echo "tests done"
cd /tmp && export TMPDIR=/tmp
SKS_BENCH_KERNELS=join,range timeout -k 10 200 python3 $R/tools/bench_pairs.py 1000 5 family > $O/pairs_family.txt 2>&1
SKS_BENCH_KERNELS=join,range timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/tools/bench_pairs.py 1000 3 family > $O/pairs_traced.txt 2>&1
SKS_BENCH_KERNELS=join,range timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD --output-format csv -d $O/p1 -o run -- python3 $R/tools/bench_pairs.py 1000 1 family > $O/p1.log 2>&1
SKS_BENCH_KERNELS=join,range timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $O/p2 -o run -- python3 $R/tools/bench_pairs.py 1000 1 family > $O/p2.log 2>&1
echo "counters done"
cd $R
timeout -k 10 300 python3 bench.py --no-sweep --no-e2e --no-c3-sharded --no-cpu-baseline > $O/bench.json 2> $O/bench.err
echo "bench done"
