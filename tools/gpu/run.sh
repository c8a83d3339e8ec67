#!/bin/bash
# The GPU-box entry point for every recorded measurement (run from gpurun:
#   gpurun -- bash tools/gpu/run.sh <task> [args]).  Outputs go to
# gpurun_out/<tag>/; each GPU step has its own time limit and the first failure
# ends the script (no GPU step after a failed one).
#
#   check [tag]                  -m gpu suite, smoke(), the default bench line (the driver's round end)
#   tests [tag] [-k expr]        -m gpu tests only (optionally a -k selection)
#   bench [tag] [bench args]     one bench.py line
#   profile <round>              tools/profile_round.sh (kernel trace + PMC passes + summary)
#   trace <tag> <cmd...>         rocprofv3 kernel trace + stats of <cmd> (a python3 script or a binary),
#                                then the per-kernel timeline of its last call (tools/kernel_timeline.py)
#   ab <tag> <variants> <cmd...> <cmd> run with this tree's library and each variants/libsks_<v>.so
#                                (comma-separated, built by tools/build_variant.sh), two alternating passes
#   rehearse [tag]               bench.py under torchrun: RCCL world 1 (one call / exchange path),
#                                gloo 2 and 3 ranks sharing GPU 0
#   ranksim [tag] [worlds...]    tools/rank_sim.py (one rank of N replayed on this GPU)
#   sweep [tag]                  the reference main (bin/kmer-sketching) on 64 config-4 FASTA files under a
#                                kernel trace, and the drop-in std::function flow (tools/dropin_flow)
#   swdiag [tag] <lib dir>       the same main with the libsks.so in <lib dir> (a stamps variant from
#                                tools/build_variant.sh, its stderr kept), then a kernel trace kept whole (gz)
#   apitrace [tag] <script...>   HIP API + kernel trace of a python3 script, both CSVs kept (gz)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TASK=$1; shift
export TMPDIR=/tmp
T="timeout -k 10"

case $TASK in
check)
  O=$R/gpurun_out/${1:-check}; mkdir -p $O; cd $R
  $T 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
    || { tail -40 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
  $T 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
  tail -2 $O/smoke.log
  $T 900 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  tail -c 600 $O/bench.json ;;
tests)
  O=$R/gpurun_out/${1:-tests}; shift; mkdir -p $O; cd $R
  $T 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "$@" > $O/tests.log 2>&1 \
    || { tail -40 $O/tests.log; exit 1; }
  tail -3 $O/tests.log ;;
bench)
  O=$R/gpurun_out/${1:-bench}; shift; mkdir -p $O; cd $R
  $T 900 python3 bench.py "$@" > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  tail -c 1500 $O/bench.json ;;
profile)
  cd $R && $T 1100 bash tools/profile_round.sh "$1" ;;
trace)
  O=$R/gpurun_out/$1; shift; mkdir -p $O; cd /tmp
  case $1 in *.py) CMD=(python3 "$R/$1");; *) CMD=("$R/$1");; esac; shift
  $T 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t -o run -- "${CMD[@]}" "$@" > $O/run.log 2>&1 \
    || { tail -20 $O/run.log; exit 1; }
  f=$(find $O/t -name '*kernel_trace.csv' | head -1)
  s=$(find $O/t -name '*kernel_stats.csv' | head -1)
  python3 $R/tools/kernel_timeline.py $f > $O/timeline.txt && cp $s $O/kernel_stats.csv
  grep -v amdgpu.ids $O/run.log | tail -5; tail -40 $O/timeline.txt ;;
ab)
  O=$R/gpurun_out/$1; V=$2; shift 2; mkdir -p $O; cd $R
  for pass in 1 2; do
    for v in base ${V//,/ }; do
      if [ $v = base ]; then L=$R/spaced-kmer-sketching_amd/lib/libsks.so; else L=$R/variants/libsks_$v.so; fi
      SKS_LIB=$L $T 300 "$@" > $O/$v.$pass.txt 2>&1 || { tail -20 $O/$v.$pass.txt; exit 1; }
      grep -v amdgpu.ids $O/$v.$pass.txt | sed "s/^/$v p$pass: /" | tail -8
    done
  done ;;
rehearse)
  O=$R/gpurun_out/${1:-reh}; mkdir -p $O; cd $R
  NB="--no-sweep --no-e2e --no-cpu-baseline --no-c2 --steps 3 --warmup 1"
  $T 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --dist-rehearsal $NB > $O/bench_1rank_rccl.json 2> $O/bench_1rank_rccl.err \
    || { tail -20 $O/bench_1rank_rccl.err; exit 1; }
  echo "rccl world 1 done"
  $T 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29518 bench.py --dist-rehearsal --world1-exchange $NB > $O/bench_1rank_rccl_exchange.json \
    2> $O/bench_1rank_rccl_exchange.err || { tail -20 $O/bench_1rank_rccl_exchange.err; exit 1; }
  echo "rccl world 1 exchange path done"
  for n in 2 3; do
    SKS_BENCH_DEVICE=0 $T 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
      --master-addr 127.0.0.1 --master-port $((29540 + n)) bench.py --gpus $n --dist-backend gloo $NB \
      > $O/bench_${n}rank_gloo.json 2> $O/bench_${n}rank.err || { tail -20 $O/bench_${n}rank.err; exit 1; }
    echo "gloo $n ranks done"
  done ;;
ranksim)
  O=$R/gpurun_out/${1:-ranksim}; shift; mkdir -p $O; cd $R
  $T 600 python3 tools/rank_sim.py "$@" > $O/rank_sim.txt 2>&1 || { tail -20 $O/rank_sim.txt; exit 1; }
  grep -v amdgpu.ids $O/rank_sim.txt ;;
sweep)
  O=$R/gpurun_out/${1:-sweep}; mkdir -p $O; cd $R
  D=/tmp/sks_sweep_files
  $T 300 python3 tools/sweep_files.py $D 64 > $O/files.log 2>&1 || { tail -5 $O/files.log; exit 1; }
  cd /tmp
  $T 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t -o run -- \
    $R/spaced-kmer-sketching_amd/bin/kmer-sketching $O/out.csv $(cat $D/list.txt) > $O/run.log 2>&1 \
    || { tail -20 $O/run.log; exit 1; }
  s=$(find $O/t -name '*kernel_stats.csv' | head -1); cp $s $O/kernel_stats.csv
  f=$(find $O/t -name '*kernel_trace.csv' | head -1)
  python3 $R/tools/kernel_timeline.py --all $f > $O/timeline.txt
  rm -rf $O/t $O/out.csv
  grep "Time taken" $O/run.log | head -8; head -25 $O/timeline.txt
  $T 600 $R/spaced-kmer-sketching_amd/bin/dropin-flow 21:21,31:31,45:35,50:40 $(cat $D/list.txt) \
    > $O/dropin.json 2> $O/dropin.err || { tail -20 $O/dropin.err; exit 1; }
  cat $O/dropin.json ;;
swdiag)
  O=$R/gpurun_out/${1:-swdiag}; L=$2; mkdir -p $O; cd $R
  D=/tmp/sks_sweep_files
  $T 300 python3 tools/sweep_files.py $D 64 > $O/files.log 2>&1 || { tail -5 $O/files.log; exit 1; }
  LD_LIBRARY_PATH=$R/$L $T 300 $R/spaced-kmer-sketching_amd/bin/kmer-sketching /tmp/o.csv $(cat $D/list.txt) \
    > $O/stamps_run.log 2> $O/stamps.err || { tail $O/stamps.err; exit 1; }
  cd /tmp
  $T 400 rocprofv3 --kernel-trace --output-format csv -d $O/t -o run -- $R/spaced-kmer-sketching_amd/bin/kmer-sketching \
    /tmp/o2.csv $(cat $D/list.txt) > $O/trace_run.log 2>&1 || { tail $O/trace_run.log; exit 1; }
  f=$(find $O/t -name '*kernel_trace.csv' | head -1); gzip -c $f > $O/kernel_trace.csv.gz; rm -rf $O/t ;;
apitrace)
  O=$R/gpurun_out/${1:-apitrace}; shift; mkdir -p $O; cd /tmp
  $T 300 rocprofv3 --hip-trace --kernel-trace --output-format csv -d $O/t -o run -- python3 "$R/$1" "${@:2}" \
    > $O/run.log 2>&1 || { tail -20 $O/run.log; exit 1; }
  for f in $(find $O/t -name '*.csv'); do gzip -c $f > $O/$(basename $f).gz; done; rm -rf $O/t
  grep -v amdgpu.ids $O/run.log | tail -3 ;;
*)
  sed -n 2,26p "$0"; exit 2 ;;
esac
