"""Distinct values per 64-sketch block of config 4's sketches (family and
unrelated genomes): the work a deduplicated (value, sketch-mask) join layout
would insert / probe instead of every element.   python tools/dedup_stats.py"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spaced-kmer-sketching_amd"))
sys.path.insert(0, ROOT)
import sksffi  # noqa: E402
import bench  # noqa: E402


def main():
    n = 1000
    ctx = sksffi.Context(0)
    L = bench.C4_LEN
    seg = [0]
    for _ in range(n):
        seg.append(seg[-1] + L + 1)
    mask = sksffi.mask_generate(31, 21, 0)
    for mode in ("family", "indep"):
        buf = torch.empty(seg[-1], dtype=torch.uint8, device="cuda")
        for g in range(n):
            a, m, r = bench.c4_genome_seeds(g)
            if mode == "indep":
                a, r = 5000 + g, 0.0
            ctx.synth_bases(buf.data_ptr() + seg[g], L, a, m, r)
        buf[torch.tensor(seg[1:], device="cuda") - 1] = ord("\n")
        ss = ctx.sketch_build(buf.data_ptr(), seg[-1], seg, 31, mask, sksffi.SKS_BOTTOM_S, 10000)
        del buf
        tot = dist = 0
        per = []
        for k in range(0, n, 64):
            vals = torch.cat([torch.from_numpy(ss.sketch(i)[:, 0].view("int64")) for i in range(k, min(n, k + 64))])
            u = torch.unique(vals.cuda()).numel()
            tot += vals.numel()
            dist += u
            per.append(round(vals.numel() / u, 2))
        print(f"{mode}: elements {tot}, distinct per block {dist}, dedup factor {tot / dist:.2f}; per block {per}",
              flush=True)


if __name__ == "__main__":
    main()
