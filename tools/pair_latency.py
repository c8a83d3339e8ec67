"""Host latency of bench.py's config-4 pair step (solo path): per step, the time
from an idle GPU to the return of all_vs_all_join (host issue) and to the
synchronised end (wall).    python tools/pair_latency.py [steps]"""
import os
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
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    n = bench.C4_GENOMES
    ctx = sksffi.Context(0)
    L = bench.C4_LEN
    seg = [0]
    for _ in range(n):
        seg.append(seg[-1] + L + 1)
    buf = torch.empty(seg[-1], dtype=torch.uint8, device="cuda")
    for g in range(n):
        a, m, r = bench.c4_genome_seeds(g)
        ctx.synth_bases(buf.data_ptr() + seg[g], L, a, m, r)
    buf[torch.tensor(seg[1:], device="cuda") - 1] = ord("\n")
    mask = sksffi.mask_generate(31, 21, 0)
    ss = ctx.sketch_build(buf.data_ptr(), seg[-1], seg, 31, mask, sksffi.SKS_BOTTOM_S, bench.C4_S)
    ops = sks_dist.GpuJoinOps(ctx)
    issue, wall, first = [], [], []
    for it in range(steps + 2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        src = sks_dist.sketches_of(ss)
        t_f = time.perf_counter()
        sks_dist.all_vs_all_join(n, 1, 0, src, ops, sksffi.join_layout_log_b, device="cuda", dst=None)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        if it >= 2:
            first.append(t_f - t0)
            issue.append(t1 - t0)
            wall.append(t2 - t0)
    print(f"views {np.median(first) * 1e3:.3f} ms  issue {np.median(issue) * 1e3:.3f} ms  "
          f"wall {np.median(wall) * 1e3:.3f} ms  k_join {ctx.last_intersect_ms():.3f} ms", flush=True)


if __name__ == "__main__":
    main()
