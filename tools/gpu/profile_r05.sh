#!/bin/bash
# quick parity subset for the host-path change, then the round profile
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out/r05p
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "rccl or fused_ani or config4 or config5 or all_vs_all or invalid" > gpurun_out/r05p/tests.log 2>&1 || { tail -30 gpurun_out/r05p/tests.log; exit 1; }
tail -1 gpurun_out/r05p/tests.log
timeout -k 10 1000 bash tools/profile_round.sh r05 > gpurun_out/r05p/profile.log 2>&1 || { tail -20 gpurun_out/r05p/profile.log; exit 1; }
tail -5 gpurun_out/r05p/profile.log
