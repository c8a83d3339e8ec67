"""Sketch builds of the first G config-4 genomes (bottom-s 10000, w = 31/k = 21),
R times, for kernel traces of the sketch phase at a rank's share
(G = 128: one rank of N = 8).
    python tools/c4_sketch.py [G] [R]"""
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spaced-kmer-sketching_amd"))
sys.path.insert(0, ROOT)
import sksffi  # noqa: E402
import bench  # noqa: E402


def main():
    G = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    R = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    L = bench.C4_LEN
    ctx = sksffi.Context(0)
    seg = [0]
    for _ in range(G):
        seg.append(seg[-1] + L + 1)
    buf = torch.empty(seg[-1], dtype=torch.uint8, device="cuda")
    for g in range(G):
        a, m, r = bench.c4_genome_seeds(g)
        ctx.synth_bases(buf.data_ptr() + seg[g], L, a, m, r)
        buf[seg[g] + L] = ord("\n")
    mask = sksffi.mask_generate(31, 21, 0)
    ms = []
    for _ in range(R):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ss = ctx.sketch_build(buf.data_ptr(), seg[-1], seg, 31, mask, sksffi.SKS_BOTTOM_S, bench.C4_S)
        torch.cuda.synchronize()
        ms.append((time.perf_counter() - t0) * 1e3)
        del ss
    print(f"{G} genomes: sketch build {statistics.median(ms[1:]):.3f} ms median (all: "
          f"{[round(x, 3) for x in ms]})")


if __name__ == "__main__":
    main()
