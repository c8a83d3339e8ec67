# full GPU test suite + default bench (+ dist rehearsal on one RCCL rank)
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/full
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gputest.log 2>&1
echo "gpu tests done"
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err
echo "bench done"
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --dist-rehearsal --no-sweep --no-e2e --no-cpu-baseline > $O/rehearsal_1rank.json 2> $O/rehearsal.err
echo "rehearsal done"
