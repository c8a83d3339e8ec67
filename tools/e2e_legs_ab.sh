#!/bin/bash
# bench.py's end-to-end legs after other legs: the overlapped FASTA pipeline
# (H2D of piece p+1 under parse + sketch of piece p) must stay at the PCIe bound
# whatever streams the earlier legs took (config 3 in flight + config 2 took six
# pool streams; a normal-priority copy stream then shared the compute queue).
set -e
B="--steps 5 --warmup 1 --no-cpu-baseline --no-sweep"
timeout -k 10 200 python bench.py $B --no-pairs --no-c3-sharded --no-c2 > gpurun_out/e2e_only.json 2>gpurun_out/e2e_only.err
timeout -k 10 200 python bench.py $B --no-pairs --no-c3-sharded > gpurun_out/e2e_c2.json 2>gpurun_out/e2e_c2.err
