set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $R/gpurun_out/sp
cd $R
SKS_LIB=$R/variants/libsks_stamps.so timeout -k 10 300 python -u -m pytest tests/test_join_dedup.py -m gpu -x -q -s --timeout 200 --timeout-method thread -k "splits_u64" > gpurun_out/sp/stamps.log 2>&1
echo done
