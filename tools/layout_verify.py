"""Checks a join layout against its sketches: per block, the (value, slot)
pairs equal the sketches'; bucket starts are non-decreasing and end at the
block total; every element's bucket is its value group (bounds) and hash.
    python tools/layout_verify.py [family|indep] [reps]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spaced-kmer-sketching_amd"))
sys.path.insert(0, ROOT)
import sksffi  # noqa: E402
import bench  # noqa: E402

PHI = np.uint64(0x9E3779B97F4A7C15)


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "indep"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    n = 1000
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
        buf[seg[g] + L] = ord("\n")
    mask = sksffi.mask_generate(31, 21, 0)
    ss = ctx.sketch_build(buf.data_ptr(), seg[-1], seg, 31, mask, sksffi.SKS_BOTTOM_S, 10000)
    d, st, sz = ss.device_ptrs()
    sizes = ss.sizes().astype(np.int64)
    sk = [ss.sketch(i)[:, 0].copy() for i in range(n)]
    tot = int(sizes.sum())
    log_b = sksffi.join_layout_log_b(int(sizes.max()))
    B = 1 << log_b
    G = sksffi.join_layout_groups(log_b)
    gb = B // G
    nb = (n + 63) // 64
    bounds = torch.empty(G + 1, dtype=torch.int64, device="cuda")
    ctx.join_layout_bounds(d, st, sz, n, log_b, bounds.data_ptr())
    bh = bounds.cpu().numpy().view(np.uint64)
    print("log_b", log_b, "G", G, "bounds monotone", bool(np.all(bh[1:] >= bh[:-1])), flush=True)
    for rep in range(reps):
        lay = (torch.empty(tot, dtype=torch.int64, device="cuda"), torch.empty(tot, dtype=torch.uint8, device="cuda"),
               torch.zeros(nb * (B + 1), dtype=torch.int32, device="cuda"), torch.zeros(nb + 1, dtype=torch.int64, device="cuda"))
        mx = ctx.join_layout_build(d, st, sz, n, log_b, *(t.data_ptr() for t in lay), stat=True, total=tot,
                                   bounds=bounds.data_ptr())
        torch.cuda.synchronize()
        data = lay[0].cpu().numpy().view(np.uint64)
        ids = lay[1].cpu().numpy()
        boff = lay[2].cpu().numpy().reshape(nb, B + 1)
        bst = lay[3].cpu().numpy()
        bad = 0
        for k in range(nb):
            a, e = int(bst[k]), int(bst[k + 1])
            got = sorted(zip(data[a:e].tolist(), ids[a:e].tolist()))
            want = sorted((int(v), i - 64 * k) for i in range(64 * k, min(n, 64 * k + 64)) for v in sk[i])
            if got != want:
                bad += 1
                gs, ws = set(got), set(want)
                print(f"rep {rep} block {k}: {len(gs - ws)} extra, {len(ws - gs)} missing; extra {sorted(gs - ws)[:3]} "
                      f"missing {sorted(ws - gs)[:3]}", flush=True)
                for v, s in sorted(ws - gs)[:3]:
                    grp = int(np.searchsorted(bh, np.uint64(v), side="right")) - 1
                    hb = int((np.uint64(v) * PHI) >> np.uint64(64 - 4)) if gb == 16 else -1
                    print(f"   missing v={v:#x} slot {s}: group {grp} hash-bucket {hb} -> bucket {grp * gb + hb}",
                          flush=True)
            if boff[k, B] != e - a or np.any(np.diff(boff[k]) < 0):
                print(f"rep {rep} block {k}: bucket starts inconsistent", flush=True)
            vals = data[a:e]
            grp = np.searchsorted(bh, vals, side="right").astype(np.int64) - 1
            hb = ((vals * PHI) >> np.uint64(64 - 4)).astype(np.int64) if gb == 16 else 0
            want_b = grp * gb + hb
            got_b = np.searchsorted(boff[k], np.arange(e - a), side="right").astype(np.int64) - 1
            nbad = int((want_b != got_b).sum())
            if nbad:
                j = int(np.nonzero(want_b != got_b)[0][0])
                print(f"rep {rep} block {k}: {nbad} elements outside their bucket, e.g. pos {j} v={int(vals[j]):#x} "
                      f"id {ids[a + j]} in bucket {got_b[j]} want {want_b[j]} (bounds {int(bh[grp[j]]):#x}.."
                      f"{int(bh[grp[j] + 1]):#x})", flush=True)
        T = sksffi.intersect_sym_tiles(n)
        ref = torch.empty((n, n), dtype=torch.int32, device="cuda")
        ctx.set_intersect_kernel(sksffi.INTERSECT_MERGE)
        ctx.intersect_sym(d, st, sz, 1, n, 0, T, ref.data_ptr())
        up = torch.triu(torch.ones(n, n, dtype=torch.bool, device="cuda"))
        fails = []
        for it in range(int(os.environ.get("LV_JOINS", "8"))):
            out = torch.zeros((n, n), dtype=torch.int32, device="cuda")
            torch.cuda.synchronize()
            ctx.intersect_sym_layout(n, log_b, *(t.data_ptr() for t in lay), 0, T, out.data_ptr())
            torch.cuda.synchronize()
            diff = (out != ref) & up
            nd = int(diff.sum())
            if nd:
                idx = torch.nonzero(diff)[:4].tolist()
                fails.append((it, nd, [(i, j, int(out[i, j]), int(ref[i, j])) for i, j in idx]))
        print(f"rep {rep}: join on this layout: {len(fails)} of {it + 1} runs differ {fails[:3]}", flush=True)
        if fails and not os.path.exists(f"gpurun_out/lv/fail_{mode}.npz"):
            k = fails[0][2][0][0] // 64  # the first differing cell's row block (a diagonal tile)
            a, e = int(bst[k]), int(bst[k + 1])
            np.savez_compressed(f"gpurun_out/lv/fail_{mode}.npz", data=data[a:e], ids=ids[a:e], boff=boff[k],
                                block=k, bounds=bh, ref=ref.cpu().numpy()[64 * k:64 * k + 64, 64 * k:64 * k + 64],
                                log_b=log_b)


if __name__ == "__main__":
    main()
