"""One rank of an N-GPU config-4 all-vs-all, replayed on one GPU (no process
group): sks_dist.all_vs_all_join runs its multi-rank path for `rank` of `world`
exactly as on N GPUs — rank 0's group bounds, the rank's own layout and tiles,
then one layout per run of peers and the plan's tiles, fused ANI into pinned host
memory — except that the exchange is replaced by copying the peers' sketches out
of the full set already on this GPU (what the exchange would deliver, padded to
the same stride).  The exchange itself is not timed here (its bytes per rank are
in DESIGN.md §7).  Also times the sketch phase of the rank's genomes.
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
        _, a0, b0 = sks_dist.block_shard(n, world, 0)
        gb0 = ops.bounds(sub(a0, b0), log_b)  # rank 0's value-group bounds, as the broadcast delivers them
        torch.cuda.synchronize()
        sks_dist._broadcast = lambda t, src, world_: t.copy_(gb0)

        def fake_exchange(own, n_genomes, world_, rank, stride, ops_, mode):
            # what the exchange leaves: every rank's slot of `per` rows, the own and
            # the peers' rows filled (the rest size 0)
            full = torch.empty((world_ * per * stride,), dtype=torch.int64, device="cuda")
            full_sz = torch.zeros(world_ * per, dtype=torch.int32, device="cuda")
            for q in [rank] + sks_dist.peer_needs(n_genomes, world_, rank):
                _, a, b = sks_dist.block_shard(n_genomes, world_, q)
                if b > a:
                    ops_.pad(sub(a, b), stride, full[q * per * stride:(q + 1) * per * stride],
                             full_sz[q * per:(q + 1) * per])
            torch.cuda.synchronize()  # the "exchange" is outside the timed region

            def wait():
                return sks_dist._strided(full, full_sz, 1, stride)
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
                                               dst=None, ani_ones=ones, ani_out=hb, max_size=mx, size_bound=S)
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
