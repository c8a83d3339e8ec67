# bench.py at 2 and 3 ranks sharing GPU 0 over gloo (the N>1 code paths: block shards, tile plan,
# layout gather, packed tiles to rank 0); the driver's own N>1 runs use RCCL on separate GPUs
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/reh
mkdir -p $O
cd $R
for n in 2 3; do
  SKS_BENCH_DEVICE=0 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29540 + n)) bench.py --gpus $n --dist-backend gloo \
    --no-sweep --no-e2e --no-cpu-baseline --no-c2 --steps 3 --warmup 1 > $O/bench_${n}rank_gloo.json 2> $O/bench_${n}rank.err
  echo "rank $n done"
done
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --dist-rehearsal --no-sweep --no-e2e --no-cpu-baseline --no-c2 --steps 3 --warmup 1 \
  > $O/bench_1rank_rccl.json 2> $O/bench_1rank_rccl.err
echo "rccl world 1 done"
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29518 bench.py --dist-rehearsal --world1-exchange --no-sweep --no-e2e --no-cpu-baseline --no-c2 \
  --steps 3 --warmup 1 > $O/bench_1rank_rccl_exchange.json 2> $O/bench_1rank_rccl_exchange.err
echo "rccl world 1 exchange path done"
