# pair phase: dense ANI copy vs the tile-row pipelined form (bench pairs legs only), trace of the pipelined run
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/pab
mkdir -p $O
cd $R
A="--steps 10 --no-c2 --no-sweep --no-e2e --no-c3-sharded --no-cpu-baseline --no-pairs-wide"
timeout -k 10 300 python3 bench.py $A > $O/dense.json 2> $O/dense.err
SKS_BENCH_PIPELINED_ANI=1 timeout -k 10 300 python3 bench.py $A > $O/pipe.json 2> $O/pipe.err
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "ani_rows" > $O/tests.log 2>&1
cd /tmp && export TMPDIR=/tmp
SKS_BENCH_PIPELINED_ANI=1 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py $A > $O/pipe_traced.json 2>&1
echo done
