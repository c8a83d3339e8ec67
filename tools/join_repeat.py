"""Determinism check of the all-pairs join on config 4's sketches: the merge
kernel's matrix once, then N join calls, each compared with it (count of
differing cells, off-diagonal sum).  SKS_JOIN_HASH_LAYOUT selects the round-2
layout build.    python tools/join_repeat.py [n_calls] [family|indep]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spaced-kmer-sketching_amd"))
sys.path.insert(0, ROOT)
import sksffi  # noqa: E402
import bench  # noqa: E402


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    mode = sys.argv[2] if len(sys.argv) > 2 else "family"
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
    T = sksffi.intersect_sym_tiles(n)
    ref = torch.empty((n, n), dtype=torch.int32, device="cuda")
    ctx.set_intersect_kernel(sksffi.INTERSECT_MERGE)
    ctx.intersect_sym(d, st, sz, 1, n, 0, T, ref.data_ptr())
    ctx.set_intersect_kernel(int(os.environ.get("JR_KERNEL", sksffi.INTERSECT_JOIN)))
    out = torch.empty((n, n), dtype=torch.int32, device="cuda")
    bad = 0
    for c in range(calls):
        ctx.intersect_sym(d, st, sz, 1, n, 0, T, out.data_ptr())
        torch.cuda.synchronize()
        diff = int((out != ref).sum())
        if diff:
            bad += 1
            idx = torch.nonzero(out != ref)[:4].tolist()
            print(f"call {c}: {diff} cells differ, e.g. {[(i, j, int(out[i, j]), int(ref[i, j])) for i, j in idx]}",
                  flush=True)
    print(f"kernel {os.environ.get('JR_KERNEL', 'join')}, {'hash' if os.environ.get('SKS_JOIN_HASH_LAYOUT') else 'grouped'} layout, {mode}: {bad} of {calls} "
          f"calls differ from the merge kernel", flush=True)


if __name__ == "__main__":
    main()
