set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/jr
mkdir -p $O
cd $R
timeout -k 10 200 python3 tools/join_repeat.py 30 family > $O/grouped_family.txt 2>&1
SKS_JOIN_HASH_LAYOUT=1 timeout -k 10 200 python3 tools/join_repeat.py 30 family > $O/hash_family.txt 2>&1
timeout -k 10 200 python3 tools/join_repeat.py 20 indep > $O/grouped_indep.txt 2>&1
echo done
SKS_JOIN_HASH_LAYOUT=1 timeout -k 10 200 python3 tools/join_repeat.py 20 indep > $O/hash_indep.txt 2>&1
JR_KERNEL=5 timeout -k 10 200 python3 tools/join_repeat.py 10 family > $O/range_family.txt 2>&1 || true
echo done2
