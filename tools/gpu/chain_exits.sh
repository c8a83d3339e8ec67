# the two-exit probe loop reproducer (tools/microbench/chain_exits.hip) on this toolchain
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $R/gpurun_out/ce
cd $R/tools/microbench
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o $R/gpurun_out/ce/chain_exits chain_exits.hip
for tb in 3 6 22; do timeout -k 10 60 $R/gpurun_out/ce/chain_exits $tb 8192 >> $R/gpurun_out/ce/chain_exits.txt 2>&1; done
/opt/rocm/bin/hipcc --version | head -2 >> $R/gpurun_out/ce/chain_exits.txt
echo done
