# repeated config-4-scale all-pairs calls of the join kernel against the merge kernel
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/jr
mkdir -p $O
cd $R
timeout -k 10 200 python3 tools/join_repeat.py 30 family > $O/family.txt 2>&1
timeout -k 10 200 python3 tools/join_repeat.py 20 indep > $O/indep.txt 2>&1
echo done
