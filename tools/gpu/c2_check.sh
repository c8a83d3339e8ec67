#!/bin/bash
# bottom-s / config-2 / all-pairs parity subset, then config-2 build latency
# (default single-round-trip path, the general path, the stamp variant) and the
# native / python all-pairs A/B
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/c2chk
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "bottom or config2 or config4 or config5 or rccl or dedup or fused_ani or all_vs_all" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 120 python3 tools/bench_c2.py 40 1 > $O/c2.txt 2>&1 || exit 1
SKS_NO_FAST_BOTTOM=1 timeout -k 10 120 python3 tools/bench_c2.py 40 1 >> $O/c2.txt 2>&1 || exit 1
SKS_LIB=$R/variants/libsks_fstamp.so timeout -k 10 120 python3 tools/bench_c2.py 4 1 >> $O/c2.txt 2>&1 || exit 1
SKS_LIB=$R/variants/libsks_fstamp.so timeout -k 10 120 python3 tools/bench_c2.py 3 64 >> $O/c2.txt 2>&1 || exit 1
grep -v amdgpu.ids $O/c2.txt
timeout -k 10 300 python3 tools/bench_ani_dest.py 15 > $O/dest.txt 2>&1
grep -v amdgpu.ids $O/dest.txt
