set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/lv
mkdir -p $O
cd $R
export LV_JOINS=${LV_JOINS:-8}
if [ -n "$LV_CHECK" ]; then export SKS_LIB=$R/spaced-kmer-sketching_amd/lib/libsks_check.so; fi
timeout -k 10 300 python3 tools/layout_verify.py indep 1 > $O/indep.txt 2>&1
timeout -k 10 300 python3 tools/layout_verify.py family 1 > $O/family.txt 2>&1
echo done
