set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $R/gpurun_out/sp
cd $R
timeout -k 10 300 python -u -m pytest tests/test_join_dedup.py -m gpu -x -v --timeout 200 --timeout-method thread -k "splits_u64 or bucket_passes" > gpurun_out/sp/tests.log 2>&1
echo done
