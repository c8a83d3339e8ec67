"""A/B timing of the scan kernel for library variants (SKS_LIB=...).
Prints median scan_ms over N builds; one process per variant.
  python tools/bench_scan.py [n_bytes] [reps] [segments]
segments > 1 cuts the bytes into that many genomes (config 4: 1000 x 5 Mb)."""
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spaced-kmer-sketching_amd"))
import sksffi  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 3_000_000_000
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 7
    nseg = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    ctx = sksffi.Context(0)
    buf = torch.empty(n + 1, dtype=torch.uint8, device="cuda")
    ctx.synth_bases(buf.data_ptr(), n, 3)
    seg = [n * i // nseg for i in range(nseg)] + [n + 1]
    for s in seg[1:]:
        buf[s - 1] = ord("\n")
    mask = sksffi.mask_generate(31, 21, 0)
    res = {}
    for kind, param in ((sksffi.SKS_FRAC_MOD, 1000), (sksffi.SKS_BOTTOM_S, 10000)):
        ms = []
        for _ in range(reps):
            ss = ctx.sketch_build(buf.data_ptr(), n + 1, seg, 31, mask, kind, param)
            ms.append(ctx.timings()["scan_ms"])
            sz = int(ss.sizes()[0])
            del ss
        med = statistics.median(ms[1:])
        res["frac" if kind == 0 else "bottom"] = (round(med, 4), round(min(ms[1:]), 4), sz,
                                                  round(n / med / 1e6, 1))
    print(os.environ.get("SKS_LIB", "default"), f"segs={nseg}", res, "(median ms, min ms, size0, "
          "Gwin/s)", flush=True)


if __name__ == "__main__":
    main()
