"""Config-4 pair phase (1000 x 5 Mb, bottom-s 10000, one rank) by where the
ANI goes: timed per step (sync to sync) for the counts only (dense), the join
with fused ANI into device memory (+ an 8 MB copy to pinned host memory), into
coarse- and fine-grained sks_host_alloc memory and into a torch pinned tensor.
    python tools/bench_ani_dest.py [reps] [w k]   (w > 32: 128-bit k-mers)"""
import os
import statistics
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spaced-kmer-sketching_amd"))
sys.path.insert(0, ROOT)
import sksffi  # noqa: E402
import sks_dist  # noqa: E402
import bench  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    w, k = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (31, 21)
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
    mask = sksffi.mask_generate(w, k, 0)
    ones = bin(mask).count("1") // 2
    ss = ctx.sketch_build(buf.data_ptr(), seg[-1], seg, w, mask, sksffi.SKS_BOTTOM_S, bench.C4_S)
    ops = sks_dist.GpuJoinOps(ctx, ew=2 if w > 32 else 1)
    src = sks_dist.sketches_of(ss, ew=ops.ew)
    mx = int(ss.sizes().max())
    print("sizes min", int(ss.sizes().min()), "max", mx, "w", w, "k", k, flush=True)
    dev = torch.zeros((n, n), dtype=torch.float64, device="cuda")
    pinned = torch.zeros(n * n, dtype=torch.float64, pin_memory=True)
    nc = sksffi.HostBuffer(n * n * 8, coherent=False)
    co = sksffi.HostBuffer(n * n * 8, coherent=True)

    def run(label, fn):
        ms = []
        for _ in range(reps + 1):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ms.append((time.perf_counter() - t0) * 1e3)
        print(f"{label:34s} median {statistics.median(ms[1:]):.3f} ms  min {min(ms[1:]):.3f}", flush=True)

    def avj(**kw):
        return sks_dist.all_vs_all_join(n, 1, 0, src, ops, sksffi.join_layout_log_b, device="cuda", dst=None,
                                        max_size=mx, size_bound=bench.C4_S, **kw)
    def interleaved(cases):  # alternate the cases rep by rep (clock drift hits all alike)
        ms = {lab: [] for lab, _ in cases}
        for _ in range(reps + 1):
            for lab, fn in cases:
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                fn()
                torch.cuda.synchronize()
                ms[lab].append((time.perf_counter() - t0) * 1e3)
        for lab, _ in cases:
            v = ms[lab][1:]
            print(f"{lab:34s} median {statistics.median(v):.3f} ms  min {min(v):.3f}", flush=True)

    def py(**kw):
        ops.no_native = True
        try:
            avj(**kw)
        finally:
            ops.no_native = False
    interleaved([("counts only (native, packed)", lambda: avj()),
                 ("counts only (python, dense)", lambda: py()),
                 ("fused ANI -> host coarse (native)", lambda: avj(ani_ones=ones, ani_out=nc)),
                 ("fused ANI -> host coarse (python)", lambda: py(ani_ones=ones, ani_out=nc))])
    run("fused ANI -> device", lambda: avj(ani_ones=ones, ani_out=dev))
    run("fused ANI -> device + 8 MB copy", lambda: (avj(ani_ones=ones, ani_out=dev),
                                                    pinned.copy_(dev.view(-1), non_blocking=True)))
    run("fused ANI -> host, coarse-grained", lambda: avj(ani_ones=ones, ani_out=nc))
    run("fused ANI -> host, fine-grained", lambda: avj(ani_ones=ones, ani_out=co))
    run("fused ANI -> torch pinned", lambda: avj(ani_ones=ones, ani_out=pinned))
    run("8 MB copy alone", lambda: pinned.copy_(dev.view(-1), non_blocking=True))
    want = dev.cpu().numpy().reshape(-1)
    for lab, a in (("coarse", nc.array), ("fine", co.array), ("pinned", pinned.numpy())):
        print(lab, "equal to device:", bool(np.array_equal(a, want)))


if __name__ == "__main__":
    main()
