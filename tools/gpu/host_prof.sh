#!/bin/bash
# host cost of the pair step (cProfile) and the layout placement's phase stamps
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/hp
mkdir -p $O
cd $R
timeout -k 10 300 python3 tools/pair_host_profile.py 60 > $O/host.txt 2>&1 || { tail -20 $O/host.txt; exit 1; }
grep -v amdgpu.ids $O/host.txt | head -80
timeout -k 10 400 bash tools/gpu/layout_stamps.sh > $O/ls.txt 2>&1 || exit 1
grep -h "stamps" $R/gpurun_out/stamps/*.txt | tail -6
