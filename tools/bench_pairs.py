"""A/B of the all-pairs intersection kernels on config 4 (1000 x 5 Mb, bottom-s
10000) or config 5's 200 genomes: sketches once, then times sks_intersect_sym
over all tiles per kernel (median of reps) and checks the matrices agree;
"onecall" (SKS_BENCH_KERNELS=join,onecall) times sks_all_pairs_ani's counts
(layout + every tile in one native call, no host round trip) sync to sync.
    python tools/bench_pairs.py [n_genomes] [reps] [family|indep|same] [w]"""
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spaced-kmer-sketching_amd"))
sys.path.insert(0, ROOT)
import sksffi  # noqa: E402
import bench  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    mode = sys.argv[3] if len(sys.argv) > 3 else "family"  # family | indep | same
    w = int(sys.argv[4]) if len(sys.argv) > 4 else 31  # 45: config 4's 128-bit leg (k = 30)
    ctx = sksffi.Context(0)
    L = bench.C4_LEN
    seg = [0]
    for _ in range(n):
        seg.append(seg[-1] + L + 1)
    buf = torch.empty(seg[-1], dtype=torch.uint8, device="cuda")
    for g in range(n):
        a, m, r = bench.c4_genome_seeds(g)
        if mode == "indep":
            a, r = 5000 + g, 0.0
        elif mode == "same":
            a, r = 100, 0.0
        ctx.synth_bases(buf.data_ptr() + seg[g], L, a, m, r)
        buf[seg[g] + L] = ord("\n")
    mask = sksffi.mask_generate(w, 21 if w == 31 else w - 15, 0)
    ss = ctx.sketch_build(buf.data_ptr(), seg[-1], seg, w, mask, sksffi.SKS_BOTTOM_S, 10000)
    data, starts, sizes = ss.device_ptrs()
    ew = ss.elem_words
    T = sksffi.intersect_sym_tiles(n)
    ref = None
    kernels = (("merge", sksffi.INTERSECT_MERGE), ("join", sksffi.INTERSECT_JOIN)) if ew == 1 else \
        (("join", sksffi.INTERSECT_JOIN),)
    kernels = kernels + (("onecall", None),)
    only = os.environ.get("SKS_BENCH_KERNELS", "merge,join")
    kernels = tuple(x for x in kernels if x[0] in only.split(","))
    for name, k in kernels:
        out = torch.empty((n, n), dtype=torch.int32, device="cuda")
        ms = []
        if name == "onecall":
            import time
            import sks_dist
            hs = ss.sizes()
            cnt = torch.empty(T * 4096, dtype=torch.int32, device="cuda")
            for _ in range(reps + 1):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                ctx.all_pairs_ani(data, starts, sizes, n, int(hs.max()), int(hs.sum()), 0, 0, cnt.data_ptr(), 0,
                                  elem_words=ew)
                torch.cuda.synchronize()
                ms.append((time.perf_counter() - t0) * 1e3)
            out.zero_()
            sks_dist.place_tiles(out, sks_dist._all_tiles((n + 63) // 64), cnt.view(T, 64, 64), n)
        else:
            ctx.set_intersect_kernel(k)
            for _ in range(reps + 1):
                ctx.intersect_sym(data, starts, sizes, ew, n, 0, T, out.data_ptr())
                ms.append(ctx.last_intersect_ms())
        got = out.cpu()
        if ref is None:
            ref = got
        same = bool(torch.equal(ref, got))
        print(f"{name:6s} {mode:6s} n={n} median {statistics.median(ms[1:]):.3f} ms  min {min(ms[1:]):.3f}"
              f"  equal_to_merge={same}  offdiag_sum={int(got.sum() - got.diag().sum())}",
              flush=True)


if __name__ == "__main__":
    main()
