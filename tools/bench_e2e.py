"""Diagnostics of bench.py's config-3 end-to-end legs (FASTA image in pinned
host memory -> H2D -> device parse -> sketch): the serial and overlapped
timings of bench.run_end_to_end, then the overlapped step once more with host
timestamps per piece (copy wait, parse, sketch, export, free) and the copy
stream's own event time per piece, to see where the overlap is lost.
    python tools/bench_e2e.py [steps] [c2]   (c2: run bench's config-2 leg first)"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spaced-kmer-sketching_amd"))
sys.path.insert(0, ROOT)
import sksffi  # noqa: E402
import bench  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    ctx = sksffi.Context(0)
    mask = sksffi.mask_generate(bench.W, bench.K, bench.MASK_SEED)
    buf, n_bytes = bench.make_c3(ctx, seed_base=3)
    if "c2" in sys.argv[2:]:
        bench.run_c2(ctx, mask, steps=4, warmup=1, inflight=3)
    res = bench.run_end_to_end(ctx, mask, buf, steps)
    print("serial ms", round(res["ms"], 2), {k: round(v, 2) for k, v in res["ms_phases"].items()},
          "overlapped ms", round(res["overlapped"]["ms"], 2), flush=True)

    # the overlapped step, instrumented (same cuts and buffers as bench)
    contig_starts, _, _ = bench.c3_layout()
    parts = []
    nl = torch.full((bench.C3_CONTIG_LEN // 80, 1), ord("\n"), dtype=torch.uint8, device="cuda")
    for i, s0 in enumerate(contig_starts):
        hdr = torch.tensor(list(f">syn_3_{i}\n".encode()), dtype=torch.uint8, device="cuda")
        body = buf[s0:s0 + bench.C3_CONTIG_LEN].view(-1, 80)
        parts += [hdr, torch.cat([body, nl], dim=1).reshape(-1)]
    dev_fa = torch.cat(parts)
    host = torch.empty(dev_fa.numel(), dtype=torch.uint8, pin_memory=True)
    host.copy_(dev_fa)
    del dev_fa, parts
    arr = host.numpy()
    import numpy as np
    heads = np.flatnonzero(arr == ord(">"))
    total = arr.size
    cuts = [0]
    for p in range(1, 8):
        j = np.searchsorted(heads, total * p // 8)
        if j < len(heads) and heads[j] > cuts[-1]:
            cuts.append(int(heads[j]))
    cuts.append(total)
    lens = [cuts[i + 1] - cuts[i] for i in range(len(cuts) - 1)]
    slots = [torch.empty(max(lens), dtype=torch.uint8, device="cuda") for _ in range(2)]
    rec = torch.empty(max(lens) + 1, dtype=torch.uint8, device="cuda")
    cs = torch.cuda.Stream()
    ws = torch.cuda.Stream()  # the instrumented context's own stream (free_on_stream)
    main_ctx = ctx
    sctx = sksffi.Context(0, ws.cuda_stream)
    ev_b = [torch.cuda.Event(enable_timing=True) for _ in lens]
    ev_e = [torch.cuda.Event(enable_timing=True) for _ in lens]
    for free_mode, ctx in (("free", main_ctx), ("free", sctx), ("free_on_stream", sctx),
                           ("keep", sctx)):
        for rep in range(2):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            rows, keep = [], []

            def h2d(p):
                with torch.cuda.stream(cs):
                    ev_b[p].record(cs)
                    slots[p % 2][:lens[p]].copy_(host[cuts[p]:cuts[p + 1]], non_blocking=True)
                    ev_e[p].record(cs)
            h2d(0)
            for p in range(len(lens)):
                if p + 1 < len(lens):
                    h2d(p + 1)
                a = time.perf_counter()
                ev_e[p].synchronize()
                b = time.perf_counter()
                nb, _ = ctx.fasta_parse_device(slots[p % 2].data_ptr(), lens[p], rec.data_ptr(), lens[p] + 1)
                c = time.perf_counter()
                ss = ctx.sketch_build(rec.data_ptr(), nb, [0, nb], bench.W, mask, sksffi.SKS_FRAC_MOD,
                                      bench.C3_FRAC)
                d = time.perf_counter()
                int(ss.sizes()[0])
                e = time.perf_counter()
                if free_mode == "free":
                    ss.free()
                elif free_mode == "free_on_stream":
                    ss.free(ws.cuda_stream)
                else:
                    keep.append(ss)
                f = time.perf_counter()
                rows.append((p, (b - a) * 1e3, (c - b) * 1e3, (d - c) * 1e3, (e - d) * 1e3, (f - e) * 1e3))
            torch.cuda.synchronize()
            tot = (time.perf_counter() - t0) * 1e3
            keep.clear()
            torch.cuda.synchronize()
            copy_ms = [ev_b[p].elapsed_time(ev_e[p]) for p in range(len(lens))]
            print(f"[{free_mode} {'null-stream ctx' if ctx is main_ctx else 'stream ctx'} rep {rep}] total {tot:.1f} ms; copy-stream ms per piece "
                  f"{[round(x, 1) for x in copy_ms]}", flush=True)
            for r in rows:
                print("   piece %d: wait-copy %.2f parse %.2f sketch %.2f sizes %.2f free %.2f" % r, flush=True)


if __name__ == "__main__":
    main()
