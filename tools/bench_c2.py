"""Config-2 single-build latency: one 5 Mb genome, bottom-s s=10000, w=31/k=21.
Prints wall ms per build and the library's own scan / post GPU times.
  python tools/bench_c2.py [reps] [genomes]   (SKS_NO_FUSED_BOTTOM=1: unfused post path)
genomes > 1: that many 5 Mb genomes in one build (the batched form)."""
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spaced-kmer-sketching_amd"))
import sksffi  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    L = 5_000_000
    n = k * (L + 1) - 1
    ctx = sksffi.Context(0)
    buf = torch.empty(n + 1, dtype=torch.uint8, device="cuda")
    seg = [0]
    for g in range(k):
        ctx.synth_bases(buf.data_ptr() + seg[-1], L, 2 + g)
        buf[seg[-1] + L] = ord("\n")
        seg.append(seg[-1] + L + 1)
    torch.cuda.synchronize()
    mask = sksffi.mask_generate(31, 21, 0)
    wall, scan, post = [], [], []
    for _ in range(reps):
        t0 = time.perf_counter()
        ss = ctx.sketch_build(buf.data_ptr(), n + 1, seg, 31, mask, sksffi.SKS_BOTTOM_S, 10000)
        wall.append((time.perf_counter() - t0) * 1e3)
        t = ctx.timings()
        scan.append(t["scan_ms"])
        post.append(t["post_ms"])
        del ss
    med = lambda x: round(statistics.median(x[2:]), 4)
    print(f"genomes={k} fused={'no' if os.environ.get('SKS_NO_FUSED_BOTTOM') else 'yes'} wall_ms={med(wall)} "
          f"scan_ms={med(scan)} post_ms={med(post)}", flush=True)


if __name__ == "__main__":
    main()
