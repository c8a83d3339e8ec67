# default bench line (the driver's command) with this round's profiles in the tree
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $R/gpurun_out/r04
cd $R
timeout -k 10 400 python3 bench.py > gpurun_out/r04/bench_n1.json 2> gpurun_out/r04/bench_n1.err
echo bench done
