# placement stamps (pass reasons) + layout/join parity subset + whole-call and kernel times
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $R/gpurun_out/pl
cd $R
timeout -k 10 400 python -u -m pytest tests/test_join_dedup.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "dedup or join or layout or tiled or adversarial" > gpurun_out/pl/tests.log 2>&1
echo tests ok
bash tools/gpu/layout_stamps.sh
rm -f gpurun_out/pt/times.txt gpurun_out/pv/summary.txt
bash tools/gpu/pairs_times.sh "$@"
