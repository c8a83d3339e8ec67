set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $R/gpurun_out/ao
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_rccl.py -m gpu -x -q --timeout 120 --timeout-method thread -k "ani_rows or all_vs_all or join_layout" > gpurun_out/ao/tests.log 2>&1
echo tests ok
timeout -k 10 300 python3 bench.py --steps 10 --no-c2 --no-sweep --no-e2e --no-c3-sharded --no-cpu-baseline > gpurun_out/ao/bench.json 2> gpurun_out/ao/bench.err
echo bench ok
