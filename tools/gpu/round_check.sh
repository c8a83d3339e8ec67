#!/bin/bash
# the driver's round-end sequence on one GPU: the -m gpu suite, smoke(), the
# default bench line; outputs in gpurun_out/<tag>/; stops at the first failure
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-round}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
  || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 900 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -c 600 $O/bench.json
