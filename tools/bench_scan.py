"""A/B timing of the config-3 scan kernel for library variants (SKS_LIB=...).
Prints median scan_ms over N builds; one process per variant."""
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
    ctx = sksffi.Context(0)
    buf = torch.empty(n + 1, dtype=torch.uint8, device="cuda")
    ctx.synth_bases(buf.data_ptr(), n, 3)
    buf[n] = ord("\n")
    mask = sksffi.mask_generate(31, 21, 0)
    res = {}
    for kind, param in ((sksffi.SKS_FRAC_MOD, 1000), (sksffi.SKS_BOTTOM_S, 10000)):
        ms = []
        for _ in range(reps):
            ss = ctx.sketch_build(buf.data_ptr(), n + 1, [0, n + 1], 31, mask, kind, param)
            ms.append(ctx.timings()["scan_ms"])
            sz = int(ss.sizes()[0])
            del ss
        res["frac" if kind == 0 else "bottom"] = (statistics.median(ms[1:]), min(ms[1:]), sz)
    print(os.environ.get("SKS_LIB", "default"), res, flush=True)


if __name__ == "__main__":
    main()
