"""Config-3 scan time vs scan grid size (sks_ctx_set_scan_grid): the grid the
occupancy query gives (4 workgroups per CU) against larger ones."""
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spaced-kmer-sketching_amd"))
import sksffi  # noqa: E402


def main():
    n = 3_000_000_000
    ctx = sksffi.Context(0)
    buf = torch.empty(n + 1, dtype=torch.uint8, device="cuda")
    ctx.synth_bases(buf.data_ptr(), n, 3)
    buf[n] = ord("\n")
    mask = sksffi.mask_generate(31, 21, 0)
    ref = None
    for grid in [0, 5120, 10240, 20480, 40960, 81920]:
        ctx.set_scan_grid(grid)
        for kind, param in ((sksffi.SKS_FRAC_MOD, 1000), (sksffi.SKS_BOTTOM_S, 10000)):
            ms = []
            for _ in range(5):
                ss = ctx.sketch_build(buf.data_ptr(), n + 1, [0, n + 1], 31, mask, kind, param)
                ms.append(ctx.timings()["scan_ms"])
                sz = int(ss.sizes()[0])
                del ss
            print(grid, "frac" if kind == sksffi.SKS_FRAC_MOD else "bottom",
                  round(statistics.median(ms[1:]), 3), round(min(ms[1:]), 3), sz, flush=True)


if __name__ == "__main__":
    main()
