# GPU suite (or a -k subset), then a bench line; usage: check.sh TAG [pytest -k expr] [bench args...]
# writes gpurun_out/TAG/{tests.log,bench.json,bench.err}; stops at the first failing step
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-chk}; K=${2:-}; shift 2 || true
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
if [ -n "$K" ]; then KA=(-k "$K"); else KA=(); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread "${KA[@]}" > $O/tests.log 2>&1
echo "tests: $(tail -1 $O/tests.log)"
timeout -k 10 600 python3 bench.py "$@" > $O/bench.json 2> $O/bench.err
echo "bench done"
