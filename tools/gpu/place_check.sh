# layout/join parity (one process, each step under its own limit), then kernel times per variant
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $R/gpurun_out/pl
cd $R
timeout -k 10 400 python -u -m pytest tests/test_join_dedup.py tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "dedup or join or layout or tiled or adversarial" > gpurun_out/pl/tests.log 2>&1
echo tests ok
timeout -k 10 400 python -u -m pytest tests/test_scale.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pl/tests_scale.log 2>&1
echo scale ok
bash tools/gpu/place_variants.sh "$@"
