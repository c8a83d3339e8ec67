"""One rank of an N-GPU config-4 all-vs-all, replayed on one GPU (no process
group): sks_dist.all_vs_all_join runs its multi-rank path for `rank` of `world`
exactly as on N GPUs — the group bounds from the mask, the rank's own export,
layout and tiles, then one layout of the own and peer rows and the plan's cross
tiles, fused ANI into pinned host memory — except that the exchange itself is
replaced: the peers' padded rows (what the exchange delivers, the peers' own
exports) are prepared once outside the timed calls, and each call writes only
the rank's own slot (its export, as on N GPUs) and hands over the buffer.  The
exchange's transfer is not timed here (its bytes per rank are in DESIGN.md §7).
Also times the sketch phase of the rank's genomes.
    python tools/rank_sim.py [world ...]      (default 2 4 8)
Prints, per world: every rank's pair-step time (median of reps) and the max."""
import os
import statistics
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spaced-kmer-sketching_amd"))
sys.path.insert(0, ROOT)
import sksffi  # noqa: E402
import sks_dist  # noqa: E402
import bench  # noqa: E402

TILE = sks_dist.TILE


def main():
    # "trace W R": only rank R of world W, 10 calls (for a kernel trace)
    trace = sys.argv[1:2] == ["trace"]
    worlds = [int(sys.argv[2])] if trace else ([int(x) for x in sys.argv[1:]] or [2, 4, 8])
    only_rank = int(sys.argv[3]) if trace else None
    n, L, S = bench.C4_GENOMES, bench.C4_LEN, bench.C4_S
    ctx = sksffi.Context(0)
    seg = [0]
    for _ in range(n):
        seg.append(seg[-1] + L + 1)
    buf = torch.empty(seg[-1], dtype=torch.uint8, device="cuda")
    for g in range(n):
        a, m, r = bench.c4_genome_seeds(g)
        ctx.synth_bases(buf.data_ptr() + seg[g], L, a, m, r)
        buf[seg[g] + L] = ord("\n")
    mask = sksffi.mask_generate(31, 21, 0)
    ones = bin(mask).count("1") // 2
    full = ctx.sketch_build(buf.data_ptr(), seg[-1], seg, 31, mask, sksffi.SKS_BOTTOM_S, S)
    allsk = sks_dist.sketches_of(full)
    ops = sks_dist.GpuJoinOps(ctx)
    hb = sksffi.HostBuffer(n * n * 8)

    def sub(g0, g1):
        return sks_dist.Sketches(allsk.data, allsk.sizes[g0:g1], 1, starts=allsk.starts[g0:g1])

    log_b = sksffi.join_layout_log_b(S)
    ref = sksffi.HostBuffer(n * n * 8)
    sks_dist.all_vs_all_join(n, 1, 0, allsk, ops, sksffi.join_layout_log_b, device="cuda", dst=None,
                             ani_ones=ones, ani_out=ref, max_size=int(full.sizes().max()), size_bound=S)
    torch.cuda.synchronize()
    for world in worlds:
        hb.array[:] = -1.0
        per = sks_dist.block_shard(n, world, 0)[0] * TILE
        # every rank's padded rows, as the peers' exports produce them (prepared
        # once, outside the timed calls); per rank the sizes of the rows its
        # exchange would leave filled (its own and its peers'; the rest size 0)
        xbuf = torch.empty((world * per * S,), dtype=torch.int64, device="cuda")
        full_sz_all = torch.zeros(world * per, dtype=torch.int32, device="cuda")
        for q in range(world):
            _, a, b = sks_dist.block_shard(n, world, q)
            if b > a:
                ops.pad(sub(a, b), S, xbuf[q * per * S:(q + 1) * per * S], full_sz_all[q * per:(q + 1) * per])
        rank_sz = {}
        for r in range(world):
            keep = torch.zeros(world * per, dtype=torch.bool, device="cuda")
            for q in [r] + sks_dist.peer_needs(n, world, r):
                keep[q * per:(q + 1) * per] = True
            rank_sz[r] = torch.where(keep, full_sz_all, torch.zeros_like(full_sz_all))
        torch.cuda.synchronize()

        def fake_exchange(own, n_genomes, world_, rank, stride, ops_, mode):
            # the rank's own slot: its export, exactly as the real exchange writes
            # it before sending; the peers' rows are already in place
            sz = rank_sz[rank]
            ops_.pad(own, stride, xbuf[rank * per * stride:(rank + 1) * per * stride], sz[rank * per:(rank + 1) * per])

            def wait():
                return sks_dist._strided(xbuf, sz, 1, stride)
            return wait
        sks_dist._exchange_start = fake_exchange
        times, sketch_ms = [], []
        for rank in range(world):
            if only_rank is not None and rank != only_rank:
                continue
            _, g0, g1 = sks_dist.block_shard(n, world, rank)
            mine = sub(g0, g1)
            mx = int(full.sizes()[g0:g1].max()) if g1 > g0 else 0
            ms = []
            for it in range(10 if trace else 8):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                res = sks_dist.all_vs_all_join(n, world, rank, mine, ops, sksffi.join_layout_log_b, device="cuda",
                                               dst=None, ani_ones=ones, ani_out=hb, max_size=mx, size_bound=S,
                                               bounds_mask=mask)
                torch.cuda.synchronize()
                ms.append((time.perf_counter() - t0) * 1e3)
            res.check_layouts()
            times.append(statistics.median(ms[2:]))
            # the rank's sketch phase: its genomes in one build
            sk = []
            for it in range(0 if trace else 4):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                ss = ctx.sketch_build(buf.data_ptr() + seg[g0], seg[g1] - seg[g0],
                                      [x - seg[g0] for x in seg[g0:g1 + 1]], 31, mask, sksffi.SKS_BOTTOM_S, S)
                torch.cuda.synchronize()
                sk.append((time.perf_counter() - t0) * 1e3)
                del ss
            sketch_ms.append(statistics.median(sk[1:]) if sk else 0.0)
        if trace:
            print(f"rank {only_rank} of {world}: {times[0]:.3f} ms")
            continue
        same = bool(np.array_equal(hb.array, ref.array))
        print(f"world {world}: ANI of all ranks equal to one process's: {same}")
        print(f"world {world}: pair step per rank (ms, exchange excluded) "
              f"{[round(x, 3) for x in times]}  max {max(times):.3f}; sketch phase per rank max "
              f"{max(sketch_ms):.3f} ms", flush=True)


if __name__ == "__main__":
    main()
