# PMC passes over tools/bench_pairs.py (family): the layout placement kernel's counters
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/ppm
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE" \
           "SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_IFETCH SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD"; do
  i=$((i+1))
  SKS_BENCH_KERNELS=join timeout -k 10 120 rocprofv3 --pmc $grp --output-format csv -d $O/family/p$i -o run -- python3 $R/tools/bench_pairs.py 1000 2 family > $O/family.p$i.log 2>&1
done
python3 $R/tools/pmc_by_kernel.py $O/family k_join k_gl_ > $O/family.txt
echo done
