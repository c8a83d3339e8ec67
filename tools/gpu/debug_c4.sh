set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $R/gpurun_out/dbg
cd $R
SKS_DEBUG_INTERSECT=1 timeout -k 10 300 python3 tools/debug_c4_join.py 1000 > gpurun_out/dbg/c4.txt 2>&1
echo done
