# layout/join parity subset, then k_gl_place / k_join per variant
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $R/gpurun_out/pl
cd $R
timeout -k 10 600 python -u -m pytest tests/test_join_dedup.py tests/test_gpu_parity.py tests/test_scale.py -m gpu -x -q --timeout 200 --timeout-method thread -k "dedup or join or layout or intersect or wide or sketches_tiled or adversarial or config4" > gpurun_out/pl/tests.log 2>&1
echo tests ok
bash tools/gpu/place_variants.sh "$@"
