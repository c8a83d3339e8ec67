# k_join workgroups per call (bucket groups per tile) on config 4, family and unrelated genomes
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/wgs
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for w in 0 1088 2176 4352 17408; do
  if [ $w = 0 ]; then unset SKS_JOIN_WGS; else export SKS_JOIN_WGS=$w; fi
  SKS_BENCH_KERNELS=join timeout -k 10 200 python3 $R/tools/bench_pairs.py 1000 5 family > $O/family_$w.txt 2>&1
  SKS_BENCH_KERNELS=join timeout -k 10 200 python3 $R/tools/bench_pairs.py 1000 5 indep > $O/indep_$w.txt 2>&1
done
echo done
