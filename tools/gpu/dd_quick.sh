# join/layout parity subset (the tree's library), the two-exit loop reproducer, then variant A/B
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $R/gpurun_out/dq
cd $R
timeout -k 10 500 python -u -m pytest tests/test_join_dedup.py tests/test_gpu_parity.py tests/test_scale.py -m gpu -x -q --timeout 200 --timeout-method thread -k "dedup or join or layout or intersect or wide or sketches_tiled or adversarial or config4" > gpurun_out/dq/tests.log 2>&1
echo tests ok
for tb in 3 6 22; do timeout -k 10 60 tools/microbench/chain_exits $tb 8192 >> gpurun_out/dq/chain_exits.txt 2>&1; done
bash tools/gpu/ab_variants.sh "$@"
