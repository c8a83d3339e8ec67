# config-4 pair path: join / RCCL / scale tests, bench pairs leg, 1-rank RCCL rehearsal
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/pc
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_rccl.py tests/test_scale.py -m gpu -x -q --timeout 200 --timeout-method thread -k "join or rccl or config4 or layout" > $O/gputest.log 2>&1
echo "gpu tests done"
timeout -k 10 300 python3 bench.py --no-sweep --no-e2e --no-c3-sharded --no-c2 --no-cpu-baseline > $O/bench.json 2> $O/bench.err
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --dist-rehearsal --no-sweep --no-e2e --no-c2 --no-c3-sharded --no-cpu-baseline > $O/rehearsal_1rank.json 2> $O/rehearsal.err
echo "bench done"
