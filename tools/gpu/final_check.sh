# parity subsets touched late in round 4, the pipelined-ANI bench legs, the miscompile reproducer, kernel times
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $R/gpurun_out/ao
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_join_dedup.py tests/test_rccl.py tests/test_scale.py -m gpu -x -q --timeout 150 --timeout-method thread -k "ani_rows or all_vs_all or join or layout or tiled or adversarial or config4 or dedup" > gpurun_out/ao/tests.log 2>&1
echo tests ok
timeout -k 10 300 python3 bench.py --steps 10 --no-c2 --no-sweep --no-e2e --no-c3-sharded --no-cpu-baseline > gpurun_out/ao/bench.json 2> gpurun_out/ao/bench.err
echo bench ok
bash tools/gpu/chain_exits.sh
rm -f gpurun_out/pt/times.txt gpurun_out/pv/summary.txt
bash tools/gpu/pairs_times.sh base
