# bench.py under torchrun at world 1 with the RCCL process group (every exchange path on RCCL)
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/reh
mkdir -p $O
cd $R
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --dist-rehearsal --no-sweep --no-e2e --no-cpu-baseline --no-c2 --steps 3 --warmup 1 \
  > $O/bench_1rank_rccl.json 2> $O/bench_1rank_rccl.err
echo "rccl world 1 done"
