"""Multi-GPU orchestration for all-vs-all ANI (one process per GPU).

The reference parallelises with cilk_for over files (kmer_set.cpp:124) and over
pairs (kmer_set.cpp:179) inside one process.  Here:
  * genomes are sharded across ranks (each rank sketches its own; no collective),
  * the padded per-rank sketches are all-gathered (RCCL over xGMI for "nccl"),
  * the upper-triangle 64x64 tiles of the N x N pair matrix are split evenly
    across ranks (sks_intersect_sym writes each count to both halves), and
  * the per-rank partial matrices are summed with one all-reduce.
The functions take the count kernel as a callable so the same orchestration is
exercised on CPU with gloo in tests/test_dist_cpu.py.
"""
import functools

import numpy as np
import torch
import torch.distributed as dist

TILE = 64


def _solo(world):
    """True when no exchange is needed: one rank and no process group.  A process
    group of size 1 (tests/test_rccl.py: RCCL on one GPU) takes the collective
    path, so every all-gather / all-reduce below runs on the backend."""
    return world == 1 and not (dist.is_available() and dist.is_initialized())


def genome_shard(n_genomes, world, rank):
    per = (n_genomes + world - 1) // world
    g0 = min(n_genomes, rank * per)
    return per, g0, min(n_genomes, g0 + per)


def sym_tiles(n):
    nb = (n + TILE - 1) // TILE
    return nb * (nb + 1) // 2


def tile_shard(n_tiles, world, rank):
    return rank * n_tiles // world, (rank + 1) * n_tiles // world


def sym_tile_coords(t, n):
    """(I, J) of upper-triangle tile t (row-major, I <= J) — intersect.hip sym_tile."""
    nb = (n + TILE - 1) // TILE
    i = 0
    while t >= nb - i:
        t -= nb - i
        i += 1
    return i, i + t


def gather_sketches(local, local_sizes, world):
    """local: [per, stride] int64 padded sketches; local_sizes: [per] int32."""
    if _solo(world):
        return local, local_sizes
    per, stride = local.shape
    if dist.get_backend() == "nccl":
        full = torch.empty((per * world, stride), dtype=local.dtype, device=local.device)
        full_sz = torch.empty(per * world, dtype=local_sizes.dtype, device=local.device)
        dist.all_gather_into_tensor(full, local)
        dist.all_gather_into_tensor(full_sz, local_sizes)
        return full, full_sz
    # gloo (CPU tests, single-GPU rehearsal): stage through host memory
    lc, lsc = local.cpu(), local_sizes.cpu()
    parts = [torch.empty_like(lc) for _ in range(world)]
    szs = [torch.empty_like(lsc) for _ in range(world)]
    dist.all_gather(parts, lc)
    dist.all_gather(szs, lsc)
    return torch.cat(parts).to(local.device), torch.cat(szs).to(local.device)


def sum_matrix(out):
    if dist.get_backend() == "nccl" or out.device.type == "cpu":
        dist.all_reduce(out)
        return out
    host = out.cpu()
    dist.all_reduce(host)
    out.copy_(host)
    return out


def all_vs_all(local, local_sizes, n_genomes, world, rank, count_sym, out=None):
    """Returns the full n x n int32 intersection matrix on every rank.

    count_sym(sketches, sizes, n, tile_begin, tile_end, out) must zero `out`
    and write the counts of upper-triangle tiles [tile_begin, tile_end) to
    both (i, j) and (j, i) — the contract of sks_intersect_sym.
    """
    src, src_sz = gather_sketches(local, local_sizes, world)
    t0, t1 = tile_shard(sym_tiles(n_genomes), world, rank)
    if out is None:
        out = torch.empty((n_genomes, n_genomes), dtype=torch.int32, device=local.device)
    count_sym(src, src_sz, n_genomes, t0, t1, out)
    if not _solo(world):
        sum_matrix(out)
    return out


def row_shard(n, world, rank):
    return rank * n // world, (rank + 1) * n // world


def all_vs_all_rows(local, local_sizes, n_genomes, world, rank, count_rows):
    """Row-block form of all_vs_all for sketches of any element width — (lo, hi)
    k-mers for 32 < w <= 64, which the join / merge tiles do not take: the padded
    sketches are all-gathered as in all_vs_all, rank r counts rows [r0, r1) against
    every column with count_rows(sketches, sizes, n, r0, r1, out_rows) (the contract
    of sks_intersect_all: out_rows[(i - r0) * n + j] = |S_i ∩ S_j|), and the row
    blocks are all-gathered.  Returns the full n x n int32 matrix on every rank."""
    src, src_sz = gather_sketches(local, local_sizes, world)
    r0, r1 = row_shard(n_genomes, world, rank)
    rows = torch.zeros((r1 - r0, n_genomes), dtype=torch.int32, device=local.device)
    if r1 > r0:
        count_rows(src, src_sz, n_genomes, r0, r1, rows)
    if _solo(world):
        return rows
    per = (n_genomes + world - 1) // world
    pad = torch.zeros((per, n_genomes), dtype=torch.int32, device=local.device)
    pad[: r1 - r0] = rows
    g = _gather_flat(pad.reshape(-1), world).view(world, per, n_genomes)
    return torch.cat([g[r, : row_shard(n_genomes, world, r)[1] - row_shard(n_genomes, world, r)[0]]
                      for r in range(world)])


# ---- seed sweep (BASELINE config 5) ----------------------------------------------------
# The reference sweeps (w, k) configurations serially, re-sketching every file
# per configuration (kmer-sketching.cpp:214-239 around :151-212).  Config 5 runs
# several spaced seeds over one genome collection; seeds are independent, so
# ranks shard by seed (rank r takes seeds r, r + world, ...), each rank keeps
# the whole collection resident, sketches it and computes its own all-vs-all
# matrix per seed.  The only exchange is the consensus: one all-reduce (sum)
# of the per-seed ANI matrices, divided by the number of seeds.

def seed_shard(n_seeds, world, rank):
    return list(range(rank, n_seeds, world))


def seed_sweep(n_seeds, world, rank, ani_for_seed, n_genomes, device="cpu"):
    """ani_for_seed(seed_index) -> [n_genomes, n_genomes] float64 tensor (row i =
    first set of the pair, as kmer-sketching.cpp:195-200).  Returns (consensus,
    local_seeds): the mean over all seeds of the ANI matrices, on every rank."""
    acc = torch.zeros((n_genomes, n_genomes), dtype=torch.float64, device=device)
    mine = seed_shard(n_seeds, world, rank)
    # ani_for_seed may return a future (host ANI of seed s overlapping the GPU
    # work of seed s + 1); resolve all of them, then sum in seed order
    parts = [ani_for_seed(s) for s in mine]
    for r in parts:
        acc += (r.result() if hasattr(r, "result") else r).to(device)
    if not _solo(world):
        sum_matrix(acc)
    acc /= n_seeds
    return acc, mine


# ---- tile plan, packed tiles, one receiving rank ------------------------------------------
# Each rank counts a fixed plan of upper-triangle 64x64 tiles (tile_plan): the
# tiles of its own blocks first — from its own data, while the exchange is in
# flight — then its half of every cross-rank block pair.  Counts stay packed
# ([tile][64][64] int32, 16 KB per tile) and go to ONE rank (dst), where the
# n x n matrix is assembled: no rank holds a matrix it does not need and no
# collective carries n^2 words (a dense all-reduce moves 2 (N-1)/N n^2 words
# through every rank).

def _ctx_waits_for_torch(ctx):
    """Order the context's HIP stream after work queued so far on torch's current
    stream (no-op when they are the same stream)."""
    s = _ctx_torch_stream(ctx)
    if s is not None:
        s.wait_stream(torch.cuda.current_stream())


def _torch_waits_for_ctx(ctx):
    s = _ctx_torch_stream(ctx)
    if s is not None:
        torch.cuda.current_stream().wait_stream(s)


def _ctx_torch_stream(ctx):
    h = getattr(ctx, "stream", 0) or 0
    cur = torch.cuda.current_stream()
    if h == cur.cuda_stream:
        return None
    return torch.cuda.default_stream() if h == 0 else torch.cuda.ExternalStream(h)


@functools.lru_cache(maxsize=64)
def tile_plan(n_genomes, world, rank):
    """(local, remote) int64 arrays [T, 2] of the upper-triangle tiles (I, J) that
    `rank` counts.  local: both blocks in the rank's own block range
    (block_shard), countable from its own sketches; remote: for every other rank
    q, half of the tiles pairing the two ranks' blocks (row-major over the pair,
    the lower rank takes the first half).  Every tile of the n x n upper
    triangle is in exactly one rank's plan; per-rank counts differ by at most
    one tile per rank pair (plus a short last rank)."""
    nb = (n_genomes + TILE - 1) // TILE
    bpr = block_shard(n_genomes, world, rank)[0]

    def blocks(q):
        return np.arange(min(nb, q * bpr), min(nb, (q + 1) * bpr), dtype=np.int64)

    mine = blocks(rank)
    I, J = np.meshgrid(mine, mine, indexing="ij")
    keep = I <= J
    local = np.stack([I[keep], J[keep]], axis=1) if mine.size else np.zeros((0, 2), np.int64)
    remote = [np.zeros((0, 2), np.int64)]
    for q in range(world):
        if q == rank:
            continue
        a, b = min(rank, q), max(rank, q)
        ba, bb = blocks(a), blocks(b)
        if not ba.size or not bb.size:
            continue
        I, J = np.meshgrid(ba, bb, indexing="ij")
        pairs = np.stack([I.reshape(-1), J.reshape(-1)], axis=1)
        h = (len(pairs) + 1) // 2
        remote.append(pairs[:h] if rank == a else pairs[h:])
    local, remote = local.reshape(-1, 2), np.concatenate(remote).reshape(-1, 2)
    local.flags.writeable = False  # cached: shared by every caller
    remote.flags.writeable = False
    return local, remote


def _max_over_many(xs, world, device):
    if _solo(world):
        return [int(x) for x in xs]
    t = torch.tensor([int(x) for x in xs], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [int(v) for v in t.tolist()]


def _gather_start(ts, world):
    """Starts the all-gathers of flat tensors (rank-major); returns a function
    that waits for them and returns the gathered tensors.  With RCCL the
    gathers run on the collective stream while the caller queues other work."""
    if dist.get_backend() == "nccl":
        outs, works = [], []
        for t in ts:
            out = torch.empty(world * t.numel(), dtype=t.dtype, device=t.device)
            works.append(dist.all_gather_into_tensor(out, t.contiguous(), async_op=True))
            outs.append(out)

        def finish():
            for w in works:
                w.wait()
            return outs
        return finish
    res = _gather_many(ts, world)  # gloo: through host memory, synchronously
    return lambda: res


def _gather_tiles(parts, world, dst):
    """parts: int32 [Tmax, 64, 64] (padded) of this rank -> [world, Tmax, 64, 64]
    on dst (None elsewhere), or on every rank when dst is None."""
    if dst is None:
        return _gather_flat(parts.reshape(-1), world).view((world,) + tuple(parts.shape))
    nccl = dist.get_backend() == "nccl"
    src = parts if nccl else parts.cpu()
    lst = [torch.empty_like(src) for _ in range(world)] if dist.get_rank() == dst else None
    dist.gather(src, gather_list=lst, dst=dst)
    if lst is None:
        return None
    return torch.stack(lst).to(parts.device)


_PLACE_CACHE = {}


def place_tiles(mat, tiles, parts, n):
    """Writes packed tile counts into the n x n matrix: tile (I, J) at rows
    64 I.., columns 64 J.., and mirrored when I != J (a diagonal tile holds both
    triangles).  The index maps depend only on (tiles, n): built once per
    process and device, then every step is two gathers and two scatters."""
    dev = mat.device
    tiles = np.asarray(tiles, dtype=np.int64).reshape(-1, 2)
    key = (tiles.tobytes(), n, str(dev))
    if key not in _PLACE_CACHE:
        if len(_PLACE_CACHE) > 4:
            _PLACE_CACHE.clear()
        t = torch.as_tensor(tiles, device=dev)
        ar = torch.arange(TILE, device=dev, dtype=torch.int64)
        gr = (t[:, 0:1] * TILE + ar.view(1, -1)).view(-1, TILE, 1).expand(-1, TILE, TILE)
        gc = (t[:, 1:2] * TILE + ar.view(1, -1)).view(-1, 1, TILE).expand(-1, TILE, TILE)
        ok = ((gr < n) & (gc < n)).reshape(-1)
        off = ((t[:, 0] != t[:, 1]).view(-1, 1, 1).expand(-1, TILE, TILE).reshape(-1)) & ok
        src_up = torch.nonzero(ok).view(-1)
        src_lo = torch.nonzero(off).view(-1)
        flat_up = (gr * n + gc).reshape(-1)[src_up]
        flat_lo = (gc * n + gr).reshape(-1)[src_lo]
        _PLACE_CACHE[key] = (src_up, flat_up, src_lo, flat_lo)
    src_up, flat_up, src_lo, flat_lo = _PLACE_CACHE[key]
    vals = parts.reshape(-1).to(dev)
    flat = mat.view(-1)
    flat[flat_up] = vals[src_up]
    flat[flat_lo] = vals[src_lo]
    return mat


# ---- all-vs-all over gathered join layouts ------------------------------------------------
# The join kernel's input (sks_join_layout_build) is built per 64-sketch block,
# so each rank builds the layout of its OWN block-aligned genome range, counts
# the tiles of its own blocks on it while the ranks all-gather their layouts
# (9 B per element + bucket starts, about the padded sketches' bytes; nothing
# is rebuilt on every rank), then counts its cross-rank tiles on the gathered
# layout.  Block k of the gathered layout is block k - r*bpr of rank r, so its
# start is shifted by r * (padded layout size).

def block_shard(n_genomes, world, rank):
    """(blocks per rank, g0, g1): genome range of `rank`, whole 64-sketch blocks."""
    n_blk = (n_genomes + TILE - 1) // TILE
    bpr = max(1, (n_blk + world - 1) // world)
    g0 = min(n_genomes, rank * bpr * TILE)
    return bpr, g0, min(n_genomes, g0 + bpr * TILE)


def _max_over(x, world, device):
    if _solo(world):
        return int(x)
    t = torch.tensor([int(x)], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return int(t.item())


def _gather_flat(t, world):
    return _gather_many([t], world)[0]


def _gather_many(ts, world):
    """All-gather of flat tensors, rank-major; with RCCL the gathers are queued
    together (async) and waited on once, so their latencies overlap."""
    if _solo(world):
        return list(ts)
    if dist.get_backend() == "nccl":
        outs, works = [], []
        for t in ts:
            out = torch.empty(world * t.numel(), dtype=t.dtype, device=t.device)
            works.append(dist.all_gather_into_tensor(out, t.contiguous(), async_op=True))
            outs.append(out)
        for w in works:
            w.wait()
        return outs
    res = []
    for t in ts:
        host = t.cpu()
        parts = [torch.empty_like(host) for _ in range(world)]
        dist.all_gather(parts, host)
        res.append(torch.cat(parts).to(t.device))
    return res


def _broadcast(t, src, world):
    if _solo(world):
        return t
    if dist.get_backend() == "nccl" or t.device.type == "cpu":
        dist.broadcast(t, src=src)
        return t
    host = t.cpu()
    dist.broadcast(host, src=src)
    t.copy_(host)
    return t


def layout_groups(log_b):
    """Value groups of a join layout with 2^log_b buckets (sks_join_layout_groups)."""
    return 1 << (log_b - 4) if log_b > 4 else 1


def all_vs_all_join(n_genomes, world, rank, local_max_size, local_total, log_b_for, build, count,
                    device="cpu", out=None, dst=0, bounds=None):
    """n x n int32 intersection matrix on rank `dst` (None on the others; on
    every rank when dst is None).

    build(log_b, pad, bounds) -> (data u64[], ids u8[], boff u32[], bstart u64[]):
    the join layout of this rank's block-aligned genomes (block_shard), with the
    value-group bounds `bounds` (an int64 tensor of layout_groups(log_b) + 1
    words; None: the rank's own).  Layouts joined with each other must share
    bounds: with a process group, rank 0 computes them (bounds(log_b) -> tensor)
    and broadcasts them before the builds.  pad is None
    for one rank without a process group; otherwise (cap_e, bpr), and the
    buffers must have exactly cap_e data / id entries, bpr * (B + 1) bucket
    starts and bpr + 1 block starts (entries past the rank's own blocks are never
    read), so they are all-gathered as they are.  cap_e is the largest rank's
    element total (one all-reduce carries it with the largest sketch size).
    count(n, log_b, layout, blk0, tiles, out) adds the counts of `tiles` (int64
    [T, 2] global block indices, I <= J) to out — the packed int32 [T, 64, 64],
    or the n x n int32 matrix (both halves) when out is 2-D — reading a layout
    whose block 0 is global block blk0: the contract of
    sks_intersect_layout_tiles.  One rank without a process group counts every
    tile straight into the matrix.

    The rank counts its tile_plan: its own blocks' tiles from its own layout
    while the layouts are being gathered, then its share of the cross-rank
    tiles; the packed tiles go to dst, which assembles the matrix.  The bucket
    count comes from the largest sketch (counts are exact at any: k_join cuts a
    bucket above its table into sub-chunks)."""
    bpr, g0, g1 = block_shard(n_genomes, world, rank)
    solo = _solo(world)
    max_all, cap_e = _max_over_many([local_max_size, local_total], world, device)
    log_b = log_b_for(max(max_all, 1))
    local, remote = tile_plan(n_genomes, world, rank)
    T = len(local) + len(remote)
    gb = None
    if not solo and bounds is not None:
        gb = bounds(log_b) if rank == 0 else \
            torch.empty(layout_groups(log_b) + 1, dtype=torch.int64, device=device)
        gb = _broadcast(gb, 0, world)
    lay = build(log_b, None if solo else (max(1, cap_e), bpr), gb)
    if solo:
        if out is None:
            out = torch.zeros((n_genomes, n_genomes), dtype=torch.int32, device=device)
        else:
            out.zero_()
        if T:
            count(n_genomes, log_b, lay, 0, local, out)
        return out
    plans = [tile_plan(n_genomes, world, q) for q in range(world)]
    sizes = [len(pl[0]) + len(pl[1]) for pl in plans]
    # the rank's packed tiles, padded to the largest plan: the gather's send buffer
    parts = torch.zeros((max(max(sizes), 1), TILE, TILE), dtype=torch.int32, device=device)
    cap_e = max(1, cap_e)
    finish = _gather_start(list(lay), world)
    if len(local):  # the rank's own tiles while the layouts travel
        count(n_genomes, log_b, lay, g0 // TILE, local, parts[:len(local)])
    g_data, g_ids, g_boff, g_bst = finish()
    # block k of rank r starts at r * cap_e in the gathered data
    g_bst = g_bst.view(world, bpr + 1)[:, :bpr] + \
        torch.arange(world, device=g_bst.device, dtype=torch.int64).view(world, 1) * cap_e
    g_bst = torch.cat([g_bst.reshape(-1),
                       torch.full((1,), world * cap_e, dtype=torch.int64, device=g_bst.device)])
    if len(remote):
        count(n_genomes, log_b, (g_data, g_ids, g_boff, g_bst), 0, remote, parts[len(local):T])
    gathered = _gather_tiles(parts, world, dst)
    if gathered is None:
        return None
    tiles = np.concatenate([np.concatenate(pl) for pl in plans]).reshape(-1, 2)
    got = torch.cat([gathered[q, :sizes[q]] for q in range(world)])
    if out is None:
        out = torch.zeros((n_genomes, n_genomes), dtype=torch.int32, device=device)
    else:
        out.zero_()
    return place_tiles(out, tiles, got, n_genomes)


def join_layout_fns(ctx, ss, local_sizes, device="cuda", cache=None):
    """The build / count / bounds callables of all_vs_all_join for this rank's sketches
    on the GPU: `ss` is the rank's SketchSet (None when it holds no genome),
    `local_sizes` its sizes (numpy).  build(log_b, pad) runs
    sks_join_layout_build into device buffers (kept in `cache` across calls of
    the same shape) and returns them on `device`; count(...) runs
    sks_intersect_layout_tiles (on the GPU, staging through `device` tensors
    when that is the CPU, as with gloo).  The context's stream is ordered after
    torch's current stream before its kernels and torch's after them, so a
    context on any stream works with the collectives on torch's."""
    n_local = len(local_sizes)
    nb_local = (n_local + TILE - 1) // TILE
    data, starts, sizes = ss.device_ptrs() if ss is not None else (0, 0, 0)
    tot = int(local_sizes.astype("int64").sum()) if n_local else 0
    cache = {} if cache is None else cache
    tile_cache = cache.setdefault("_tiles", {}) if isinstance(cache, dict) else {}
    keep = {}

    def bounds(log_b):
        b = torch.empty(layout_groups(log_b) + 1, dtype=torch.int64, device="cuda")
        _ctx_waits_for_torch(ctx)
        ctx.join_layout_bounds(data, starts, sizes, n_local, log_b, b.data_ptr())
        _torch_waits_for_ctx(ctx)
        keep["bounds"] = b
        return b.to(device)

    def build(log_b, pad=None, gbounds=None):
        B1 = (1 << log_b) + 1
        gb = gbounds.to("cuda").contiguous() if gbounds is not None else None
        # padded (all_vs_all_join with a process group): the send buffers
        # themselves, cap_e elements and bpr blocks, gathered as they are
        cap_e, nb = pad if pad is not None else (max(tot, 1), max(nb_local, 1))
        key = (cap_e, log_b, nb)
        if key not in cache:  # layout buffers persist across steps
            for k in [k for k in cache if k != "_tiles"]:
                del cache[k]
            cache[key] = (torch.empty(cap_e, dtype=torch.int64, device="cuda"),
                          torch.empty(cap_e, dtype=torch.uint8, device="cuda"),
                          torch.zeros(nb * B1, dtype=torch.int32, device="cuda"),
                          torch.zeros(nb + 1, dtype=torch.int64, device="cuda"))
        out = cache[key]
        _ctx_waits_for_torch(ctx)  # the buffers' previous readers (gathers, joins)
        ctx.join_layout_build(data, starts, sizes, n_local, log_b, *(t.data_ptr() for t in out), stat=False,
                              total=tot, bounds=gb.data_ptr() if gb is not None else None)
        _torch_waits_for_ctx(ctx)
        keep["gb"] = gb
        return tuple(t.to(device) for t in out)

    def count(n, log_b, lay, blk0, tiles, out):
        lay = [t.to("cuda") for t in lay]
        key = ("tiles", tiles.tobytes())  # the plan repeats every step: upload it once
        if key not in tile_cache:
            if len(tile_cache) > 8:
                tile_cache.clear()
            tile_cache[key] = torch.from_numpy(np.array(tiles, dtype=np.int32)).reshape(-1, 2).to("cuda").contiguous()
        tl = tile_cache[key]
        tgt = out if out.is_cuda else torch.zeros(out.shape, dtype=out.dtype, device="cuda")
        _ctx_waits_for_torch(ctx)
        ctx.intersect_layout_tiles(n, log_b, *(t.data_ptr() for t in lay), blk0, tl.data_ptr(), 0,
                                   tl.shape[0], out.dim() == 3, tgt.data_ptr())
        _torch_waits_for_ctx(ctx)
        keep["last"] = (lay, tl)  # alive until torch's stream is past the kernel
        if tgt is not out:
            out.copy_(tgt.cpu())
    return build, count, bounds


# ---- one genome across ranks (SURVEY §8e, config 3 strong scaling) -----------------------
# FracMinHash keeps a k-mer on its own hash, so the sketch of a genome is the
# union of the sketches of chunks cut with (w-1)-base halos: rank r scans the
# windows that start in [r*n/world, (r+1)*n/world), the chunk sets are
# all-gathered (padded to the largest) and every rank forms the sorted union.

def genome_chunk(n_bytes, w, world, rank):
    a = n_bytes * rank // world
    b = n_bytes * (rank + 1) // world
    return a, min(n_bytes, b + w - 1) if b > a else b


def sketch_genome_sharded(n_bytes, w, world, rank, build_chunk, union, device="cpu"):
    """build_chunk(a, b) -> (int64 tensor of the chunk's sorted k-mers, windows):
    shape [k] for w <= 32, [k, 2] (lo, hi) for w > 32; union(t) -> sorted distinct
    k-mers of t (same shape convention).  Returns (sketch, total windows) on
    every rank."""
    a, b = genome_chunk(n_bytes, w, world, rank)
    vals, nw = build_chunk(a, b)
    if _solo(world):
        return vals, nw
    k = vals.shape[0]
    rest = tuple(vals.shape[1:])
    kmax = max(1, _max_over(k, world, device))
    pad = torch.zeros((kmax,) + rest, dtype=torch.int64, device=device)
    pad[:k] = vals
    g = _gather_flat(pad.reshape(-1), world).view((world, kmax) + rest)
    sizes = _gather_flat(torch.tensor([k], dtype=torch.int64, device=device), world)
    keep = torch.arange(kmax, device=device).view(1, kmax) < sizes.view(world, 1)
    t = torch.tensor([nw], dtype=torch.int64, device=device)
    dist.all_reduce(t)
    return union(g[keep]), int(t.item())
