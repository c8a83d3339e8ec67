"""Debug: config-4 1000 x 5 Mb all-pairs through the solo all_vs_all_join path,
sks_intersect_sym (join) and the merge kernel; prints where they differ."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spaced-kmer-sketching_amd"))
sys.path.insert(0, ROOT)
import sksffi  # noqa: E402
import sks_dist  # noqa: E402
import bench  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
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
    d, st, sz = ss.device_ptrs()
    T = sksffi.intersect_sym_tiles(n)
    mats = {}
    for name, k in (("merge", sksffi.INTERSECT_MERGE), ("join", sksffi.INTERSECT_JOIN)):
        ctx.set_intersect_kernel(k)
        o = torch.full((n, n), -1, dtype=torch.int32, device="cuda")
        ctx.intersect_sym(d, st, sz, 1, n, 0, T, o.data_ptr())
        torch.cuda.synchronize()
        mats[name] = o.cpu().numpy()
    ctx.set_intersect_kernel(sksffi.INTERSECT_AUTO)
    res = sks_dist.all_vs_all_join(n, 1, 0, sks_dist.sketches_of(ss), sks_dist.GpuJoinOps(ctx),
                                   sksffi.join_layout_log_b, device="cuda")
    torch.cuda.synchronize()
    mats["solo"] = res.matrix.cpu().numpy()
    ctx.set_join_check(True)
    o = torch.full((n, n), -1, dtype=torch.int32, device="cuda")
    ctx.intersect_sym(d, st, sz, 1, n, 0, T, o.data_ptr())
    print("check violations", ctx.join_check_violations(), flush=True)
    ctx.set_join_check(False)
    mats["checked"] = o.cpu().numpy()
    ref = mats["merge"]
    for name, m in mats.items():
        bad = np.argwhere(m != ref)
        print(name, "sym", np.array_equal(m, m.T), "diff cells", len(bad), flush=True)
        for i, j in bad[:12]:
            print("   ", i, j, "blk", i // 64, j // 64, "got", m[i, j], "want", ref[i, j], "mirror", m[j, i])
        if len(bad):
            blk = np.unique(np.stack([bad[:, 0] // 64, bad[:, 1] // 64], 1), axis=0)
            print("    tiles", blk[:20].tolist())


if __name__ == "__main__":
    main()
