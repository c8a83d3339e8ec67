"""Join-layout statistics for config 4 (1000 x 5 Mb, bottom-s 10000): per
(block, value group) raw element counts and distinct values (the dedup
factor), from the sketches and the layout's own group bounds, on the host.
    python tools/layout_stats.py [n_genomes]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spaced-kmer-sketching_amd"))
sys.path.insert(0, ROOT)
import sksffi  # noqa: E402
import bench  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    mode = sys.argv[2] if len(sys.argv) > 2 else "family"
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
        ctx.synth_bases(buf.data_ptr() + seg[g], L, a, m, r)
    buf[torch.tensor(seg[1:], device="cuda") - 1] = ord("\n")
    mask = sksffi.mask_generate(31, 21, 0)
    ss = ctx.sketch_build(buf.data_ptr(), seg[-1], seg, 31, mask, sksffi.SKS_BOTTOM_S, bench.C4_S)
    d, st, sz = ss.device_ptrs()
    sizes = ss.sizes()
    log_b = sksffi.join_layout_log_b(int(sizes.max()))
    G = sksffi.join_layout_groups(log_b)
    b = torch.empty(G + 1, dtype=torch.int64, device="cuda")
    ctx.join_layout_bounds(d, st, sz, n, log_b, b.data_ptr())
    torch.cuda.synchronize()
    bounds = b.cpu().numpy().view(np.uint64)
    sk = [ss.sketch(i)[:, 0] for i in range(n)]
    raw, dist, fat = [], [], []
    for b0 in range(0, n, 64):
        blk = sk[b0:b0 + 64]
        gi = [np.searchsorted(bounds[1:G], s, side="right") for s in blk]
        allv = np.concatenate(blk)
        allg = np.concatenate(gi)
        per = np.stack([np.bincount(x, minlength=G) for x in gi])  # [sketch, group]
        for g in range(G):
            v = allv[allg == g]
            raw.append(len(v))
            dist.append(len(np.unique(v)))
            fat.append(int(per[:, g].max()))
    raw, dist, fat = np.array(raw), np.array(dist), np.array(fat)
    top = np.argsort(raw)[-8:]
    print("largest groups (block, group, raw, distinct, largest per-sketch count):",
          [(int(t // G), int(t % G), int(raw[t]), int(dist[t]), int(fat[t])) for t in top])
    print("groups with a sketch above 48:", int((fat > 48).sum()), "first few:",
          [(int(t // G), int(t % G), int(raw[t]), int(fat[t])) for t in np.nonzero(fat > 48)[0][:8]])
    print(f"{mode} n={n} log_b={log_b} G={G}: raw per group mean {raw.mean():.0f} max {raw.max()} "
          f"p99 {np.percentile(raw, 99):.0f} (> 2048: {(raw > 2048).sum()} of {len(raw)}); distinct mean "
          f"{dist.mean():.0f} max {dist.max()}; dedup {raw.sum() / dist.sum():.2f}x", flush=True)


if __name__ == "__main__":
    main()
