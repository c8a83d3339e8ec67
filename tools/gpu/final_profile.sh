#!/bin/bash
# the new GPU test, then the round profile of the final tree
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out/fp
timeout -k 10 300 python -u -m pytest tests/test_join_dedup.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "hint" > gpurun_out/fp/tests.log 2>&1 || { tail -30 gpurun_out/fp/tests.log; exit 1; }
tail -1 gpurun_out/fp/tests.log
timeout -k 10 1000 bash tools/profile_round.sh r05 > gpurun_out/fp/profile.log 2>&1 || { tail -20 gpurun_out/fp/profile.log; exit 1; }
tail -4 gpurun_out/fp/profile.log
