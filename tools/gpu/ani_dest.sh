# where the fused ANI goes (tools/bench_ani_dest.py); optional: layout stamps
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/ad
mkdir -p $O
cd $R
timeout -k 10 300 python3 tools/bench_ani_dest.py 10 > $O/dest.txt 2>&1
echo "dest done"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_scale.py tests/test_rccl.py -m gpu -x -q --timeout 300 --timeout-method thread -k "fused or config4 or rccl" > $O/tests.log 2>&1
echo "tests: $(tail -1 $O/tests.log)"
