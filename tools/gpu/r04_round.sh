# round 4: full GPU suite, then the round profile (traced default bench, PMC traffic, scan / pair counters)
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $R/gpurun_out/r04
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r04/gputest.log 2>&1
echo "gpu tests done"
bash tools/profile_round.sh r04 > gpurun_out/r04/profile.log 2>&1
echo "profile done"
