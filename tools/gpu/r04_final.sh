# end of round 4: full GPU suite, smoke, default bench line
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $R/gpurun_out/r04f
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r04f/gputest.log 2>&1
echo "gpu tests done"
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04f/smoke.log 2>&1
echo "smoke done"
timeout -k 10 400 python3 bench.py > gpurun_out/r04f/bench_n1.json 2> gpurun_out/r04f/bench_n1.err
echo "bench done"
