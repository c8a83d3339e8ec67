set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $R/gpurun_out/ls
cd $R
timeout -k 10 200 python3 tools/layout_stats.py 1000 family > gpurun_out/ls/family.txt 2>&1
timeout -k 10 200 python3 tools/layout_stats.py 1000 indep > gpurun_out/ls/indep.txt 2>&1
echo done
