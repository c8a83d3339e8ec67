"""Config-4 pair step (fused ANI into pinned host memory) timed right after a
sketch build and again with no build in between, alternating, to separate the
pair step's own time from the effect of the build before it (bench.py times
the former).
    python tools/pair_after_sketch.py [reps]"""
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spaced-kmer-sketching_amd"))
sys.path.insert(0, ROOT)
import sksffi  # noqa: E402
import sks_dist  # noqa: E402
import bench  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
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
    torch.cuda.synchronize()
    mask = sksffi.mask_generate(31, 21, 0)
    ones = bin(mask).count("1") // 2
    ops = sks_dist.GpuJoinOps(ctx, ew=1)
    host = sksffi.HostBuffer(n * n * 8)

    def step(ss):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        sks_dist.all_vs_all_join(n, 1, 0, sks_dist.sketches_of(ss, ew=1), ops, sksffi.join_layout_log_b,
                                 device="cuda", dst=None, ani_ones=ones, ani_out=host,
                                 max_size=int(ss.sizes().max()), size_bound=bench.C4_S, bounds_mask=mask)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3

    first, again, build = [], [], []
    ss = None
    for it in range(reps + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ss = None
        ss = ctx.sketch_build(buf.data_ptr(), seg[-1], seg, 31, mask, sksffi.SKS_BOTTOM_S, bench.C4_S)
        torch.cuda.synchronize()
        b = (time.perf_counter() - t0) * 1e3
        f = step(ss)
        a = step(ss)
        if it:
            build.append(b)
            first.append(f)
            again.append(a)
    med = lambda x: round(statistics.median(x), 3)
    print(f"sketch {med(build)} ms | pair right after the build: median {med(first)} mean "
          f"{round(statistics.mean(first), 3)} | pair again: median {med(again)} mean {round(statistics.mean(again), 3)}",
          flush=True)
    print("after build", [round(x, 3) for x in first], flush=True)
    print("again      ", [round(x, 3) for x in again], flush=True)


if __name__ == "__main__":
    main()
