"""Per-kernel timeline of one config-4 all-pairs call (the bench's pair step at
N = 1: sks_all_pairs_ani, counts only or with the fused ANI to pinned host
memory), from a rocprofv3 kernel trace of tools/bench_ani_dest-style calls.
    run:       python tools/pair_call_trace.py run [reps] [ani|counts] [w]   (under rocprofv3 --kernel-trace)
    summarize: python tools/pair_call_trace.py sum <kernel_trace.csv> [reps]
The summary prints, for the last call, each kernel's start offset from the
call's first kernel, its duration and the idle gap before it."""
import csv
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(reps, ani, w=31):
    import torch
    sys.path.insert(0, os.path.join(ROOT, "spaced-kmer-sketching_amd"))
    sys.path.insert(0, ROOT)
    import sksffi
    import sks_dist
    import bench
    n, L = bench.C4_GENOMES, bench.C4_LEN
    ctx = sksffi.Context(0)
    seg = [0]
    for _ in range(n):
        seg.append(seg[-1] + L + 1)
    buf = torch.empty(seg[-1], dtype=torch.uint8, device="cuda")
    for g in range(n):
        a, m, r = bench.c4_genome_seeds(g)
        ctx.synth_bases(buf.data_ptr() + seg[g], L, a, m, r)
        buf[seg[g] + L] = ord("\n")
    mask = sksffi.mask_generate(w, 21 if w == 31 else w - 15, 0)
    ones = bin(mask).count("1") // 2
    ss = ctx.sketch_build(buf.data_ptr(), seg[-1], seg, w, mask, sksffi.SKS_BOTTOM_S, bench.C4_S)
    src = sks_dist.sketches_of(ss)
    ops = sks_dist.GpuJoinOps(ctx, ew=ss.elem_words)
    mx = int(ss.sizes().max())
    hb = sksffi.HostBuffer(n * n * 8)
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        sks_dist.all_vs_all_join(n, 1, 0, src, ops, sksffi.join_layout_log_b, device="cuda", dst=None,
                                 max_size=mx, size_bound=bench.C4_S, ani_ones=ones if ani else None,
                                 ani_out=hb if ani else None)
        torch.cuda.synchronize()
        print(f"call {(time.perf_counter() - t0) * 1e3:.3f} ms", flush=True)


def summarize(path, reps):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # the calls' kernels: from the last k_gl_prep on
    starts = [i for i, r in enumerate(rows) if "k_gl_prep" in r["Kernel_Name"]]
    last = rows[starts[-1]:]
    t0 = int(last[0]["Start_Timestamp"])
    prev_end = t0
    for r in last:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r["Kernel_Name"].split("(")[0][-60:]
        print(f"{(s - t0) / 1e3:9.1f} us  dur {(e - s) / 1e3:8.1f} us  gap {(s - prev_end) / 1e3:7.1f} us  {name}")
        prev_end = e
    print(f"first kernel start -> last kernel end: {(prev_end - t0) / 1e3:.1f} us")


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(int(sys.argv[2]) if len(sys.argv) > 2 else 10, len(sys.argv) > 3 and sys.argv[3] == "ani",
            int(sys.argv[4]) if len(sys.argv) > 4 else 31)
    else:
        summarize(sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 10)
