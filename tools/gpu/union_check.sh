#!/bin/bash
# the one-peer-layout multi-rank path: RCCL world-1 tests, the one-rank replay at N = 2/4/8,
# and the world-1 RCCL rehearsal on the exchange path
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out/uc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "rccl or all_vs_all or fused_ani" > gpurun_out/uc/tests.log 2>&1 || { tail -30 gpurun_out/uc/tests.log; exit 1; }
tail -1 gpurun_out/uc/tests.log
timeout -k 10 400 python3 tools/rank_sim.py 2 4 8 > gpurun_out/uc/rank_sim.txt 2>&1 || { tail gpurun_out/uc/rank_sim.txt; exit 1; }
grep world gpurun_out/uc/rank_sim.txt
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29518 bench.py --dist-rehearsal --world1-exchange --no-sweep --no-e2e --no-cpu-baseline --no-c2 \
  --steps 5 --warmup 2 > gpurun_out/uc/bench_1rank_rccl_exchange.json 2> gpurun_out/uc/reh.err || { tail gpurun_out/uc/reh.err; exit 1; }
python3 -c "
import json
d=json.loads([x for x in open('gpurun_out/uc/bench_1rank_rccl_exchange.json') if x.startswith('{')][-1])
print('world-1 exchange path: pairs', d['pairs']['ms_pair_phase'], 'wide', d['pairs_wide']['ms_pair_phase'], d['pairs']['ani_mean_all_pairs'])"
