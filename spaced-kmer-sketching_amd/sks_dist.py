"""Multi-GPU orchestration for all-vs-all ANI (one process per GPU).

The reference parallelises with cilk_for over files (kmer_set.cpp:124) and over
pairs (kmer_set.cpp:179) inside one process.  Here (all_vs_all_join):
  * genomes are sharded across ranks in whole 64-sketch blocks; each rank
    sketches its own and builds the join layout of its own blocks,
  * every rank's sketches are broadcast by their owner (RCCL over xGMI for
    "nccl"), and each receiver joins its blocks with the source's as they land
    (a fixed tile plan splits the upper-triangle 64x64 tiles between ranks),
  * containment / ANI are computed per tile on the rank that counted it, and
    the packed count tiles are assembled into the n x n matrix on one rank
    only when asked.
Config 5 shards seeds (seed_sweep: one all-reduce of ANI sums) and config 3
shards genomes or one genome's chunks (sketch_genome_sharded).  The functions
take the kernels as callables so the same orchestration is exercised on CPU
with gloo in tests/test_dist_cpu.py.
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


# ---- stream ordering, packed tiles, one receiving rank ---------------------------------------
# Each rank counts a fixed plan of upper-triangle 64x64 tiles (tile_plan): the
# tiles of its own blocks first — from its own data, while the exchange is in
# flight — then its half of every cross-rank block pair.  Counts stay packed
# ([tile][64][64] int32, 16 KB per tile); when asked they go to ONE rank (dst),
# where the n x n matrix is assembled: no collective carries n^2 words.

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


_EXT_STREAMS = {}


def _ctx_torch_stream(ctx):
    h = getattr(ctx, "stream", 0) or 0
    cur = torch.cuda.current_stream()
    if h == cur.cuda_stream:
        return None
    if h == 0:
        return torch.cuda.default_stream()
    if h not in _EXT_STREAMS:  # one wrapper per HIP stream (building one per call costs host time)
        _EXT_STREAMS[h] = torch.cuda.ExternalStream(h)
    return _EXT_STREAMS[h]


def _gather_tiles(parts, world, dst):
    """parts: [Tmax, 64, 64] (padded) of this rank -> [world, Tmax, 64, 64] on dst
    (None elsewhere), or on every rank when dst is None."""
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


# ---- all-vs-all over join layouts, sketches exchanged per source rank ---------------------
# The join kernel's input (sks_join_layout_build) is built per 64-sketch block.
# Each rank owns whole blocks (block_shard), sketches them and builds the layout
# of its own blocks; it counts its own blocks' tiles on that layout at once.
# Every rank's sketches are then broadcast by their owner (all ranks issue the
# broadcasts in rank order; with RCCL they run on the collective stream), and
# as source q's sketches land, the receiver builds q's block layout and counts
# its share of the (own, q) tiles (tile_plan), while the later sources are
# still in flight.  Raw sketches travel (8 B per element, or 16 B for 128-bit
# k-mers) rather than layouts: a deduplicated layout keeps its regions at raw
# offsets (16 B per raw element with the mask), and rebuilding a peer's layout
# (~90 us for all of config 4) costs less than moving twice the bytes.  All
# layouts share rank 0's value-group bounds (broadcast first), so every pair of
# blocks is bucketed alike.  Counts stay packed per tile; containment / ANI are
# computed per tile on the rank that counted it (sks_ani_tiles); the count
# tiles are assembled into the n x n matrix only where asked (dst).

def block_shard(n_genomes, world, rank):
    """(blocks per rank, g0, g1): genome range of `rank`, whole 64-sketch blocks."""
    n_blk = (n_genomes + TILE - 1) // TILE
    bpr = max(1, (n_blk + world - 1) // world)
    g0 = min(n_genomes, rank * bpr * TILE)
    return bpr, g0, min(n_genomes, g0 + bpr * TILE)


@functools.lru_cache(maxsize=64)
def tile_plan_by_peer(n_genomes, world, rank):
    """(local, remote): local int64 [T, 2] — the upper-triangle tiles (I, J)
    with both blocks in the rank's own block range; remote — a list over ranks
    q of the tiles pairing the two ranks' blocks that `rank` counts (row-major
    over the pair, the lower rank takes the first half; I is in the lower
    rank's blocks, J in the higher's; empty for q == rank)."""
    nb = (n_genomes + TILE - 1) // TILE
    bpr = block_shard(n_genomes, world, rank)[0]

    def blocks(q):
        return np.arange(min(nb, q * bpr), min(nb, (q + 1) * bpr), dtype=np.int64)

    mine = blocks(rank)
    I, J = np.meshgrid(mine, mine, indexing="ij")
    keep = I <= J
    local = np.stack([I[keep], J[keep]], axis=1).reshape(-1, 2) if mine.size else np.zeros((0, 2), np.int64)
    remote = []
    for q in range(world):
        a, b = min(rank, q), max(rank, q)
        ba, bb = blocks(a), blocks(b)
        if q == rank or not ba.size or not bb.size:
            remote.append(np.zeros((0, 2), np.int64))
            continue
        I, J = np.meshgrid(ba, bb, indexing="ij")
        pairs = np.stack([I.reshape(-1), J.reshape(-1)], axis=1)
        h = (len(pairs) + 1) // 2
        remote.append(pairs[:h] if rank == a else pairs[h:])
    local.flags.writeable = False  # cached: shared by every caller
    for r in remote:
        r.flags.writeable = False
    return local, tuple(remote)


def tile_plan(n_genomes, world, rank):
    """(local, remote) int64 arrays [T, 2] of the upper-triangle tiles (I, J) that
    `rank` counts: its own blocks' tiles, then its share of every cross-rank
    block pair (tile_plan_by_peer, concatenated in rank order).  Every tile of
    the n x n upper triangle is in exactly one rank's plan."""
    local, remote = tile_plan_by_peer(n_genomes, world, rank)
    return local, np.concatenate(remote).reshape(-1, 2)


class Sketches:
    """A rank's sketch set as tensors: data int64 [total * ew] (sketches back to
    back), sizes int32 [n], starts int64 [n] (element index of each sketch)."""

    def __init__(self, data, sizes, ew=1, starts=None):
        self.data, self.sizes, self.ew = data, sizes, ew
        self.n = int(sizes.numel())
        if starts is None:
            starts = torch.zeros(self.n, dtype=torch.int64, device=sizes.device)
            if self.n > 1:
                starts[1:] = torch.cumsum(sizes[:-1].to(torch.int64), 0)
        self.starts = starts
        self.total = int(data.numel()) // ew


def _exchange_start(own, ns, totals, world, rank):
    """Starts one broadcast per source rank (in rank order, on every rank) of
    the source's sketches; returns wait(q) -> Sketches of rank q.  With RCCL the
    broadcasts run on the collective stream and wait(q) only orders torch's
    current stream after source q's (the host does not block); with gloo the
    data goes through host memory, synchronously."""
    ew, dev = own.ew, own.data.device
    nccl = dist.get_backend() == "nccl"
    bufs = []
    for q in range(world):
        if q == rank:
            bufs.append((own.data, own.sizes))
        else:
            bufs.append((torch.empty(max(totals[q] * ew, 1), dtype=torch.int64, device=dev if nccl else "cpu"),
                         torch.empty(max(ns[q], 1), dtype=torch.int32, device=dev if nccl else "cpu")))
    works = []
    for q in range(world):
        d, sz = bufs[q]
        nd, nz = totals[q] * ew, ns[q]
        if not nccl and q == rank:
            d, sz = d.cpu(), sz.cpu()
        ws = []
        for t, k in ((d, nd), (sz, nz)):
            if k:  # every rank knows the sizes: all skip empty sources alike
                ws.append(dist.broadcast(t[:k], src=q, async_op=nccl))
        works.append(ws)
        if not nccl:
            bufs[q] = (d, sz)

    def wait(q):
        if q == rank:
            return own
        for w in works[q]:
            if nccl and w is not None:
                w.wait()
        d, sz = bufs[q]
        if not nccl:
            d, sz = d.to(dev), sz.to(dev)
        return Sketches(d[:totals[q] * ew], sz[:ns[q]], ew)
    return wait


class JoinResult:
    """What all_vs_all_join leaves on a rank.  tiles: int64 [T, 2] (None for one
    rank without a process group, whose counts / ani are the dense n x n
    matrices); counts: packed int32 [T, 64, 64]; ani: float64 [T, 2, 64, 64]
    (both orientations, sks_ani_tiles) or dense, when asked; matrix: the n x n
    int32 counts on the assembling rank(s), else None."""

    def __init__(self):
        self.tiles = self.counts = self.ani = self.matrix = None


def _row_parts(nb, parts=6):
    """Tile-row ranges [I0, I1) of an nb x nb upper triangle with about
    T / parts tiles each (the early tile rows hold the most tiles)."""
    T = nb * (nb + 1) // 2
    target = max(1, -(-T // parts))
    out, i0, acc = [], 0, 0
    for i in range(nb):
        acc += nb - i
        if acc >= target or i == nb - 1:
            out.append((i0, i + 1))
            i0, acc = i + 1, 0
    return out


def _tiles_before(I, nb):
    """Upper-triangle tiles (row-major) before tile row I."""
    return I * nb - I * (I - 1) // 2


def all_vs_all_join(n_genomes, world, rank, mine, ops, log_b_for, device="cpu", dst=0, ani_ones=None,
                    ani_host=None, pipelined=False, max_size=None):
    """All-vs-all intersection counts (kmer_set.cpp:143-184 over the
    generate_all_pairs_from_vector list, generators.hpp:44-58), and ANI when
    ani_ones (the k of binomial_estimator) is given.

    mine: Sketches of this rank's block-aligned genomes (block_shard).
    ops: the kernels (GpuJoinOps on the GPU; a numpy restatement in the CPU
    tests): ew; bounds(src, log_b) -> group bounds tensor; build(src, log_b,
    bounds, key) -> layout (cached by key); count(n, log_b, rows, r_blk0, cols,
    c_blk0, tiles, out) — the contract of sks_intersect_layout_pair_tiles
    (tiles None: every upper-triangle tile into the dense matrix out);
    ani_matrix(counts, n, k); ani_tiles(tiles, packed, sizes, n, k).
    dst: the rank that assembles the n x n count matrix (None: none, "all":
    every rank).  ani_host (one rank, no process group): a pinned host tensor of
    n * n float64 that receives the ANI matrix (queued, not waited for);
    pipelined: count in tile-row parts and copy each part's finished ANI rows
    while later parts are counted (measured slower on config 4: DESIGN.md §6).
    Returns a JoinResult."""
    res = JoinResult()
    bpr, g0, g1 = block_shard(n_genomes, world, rank)
    solo = _solo(world)
    # the largest local sketch (max_size: known to the caller's host, e.g. from
    # SketchSet.sizes(); else one device reduction and a read-back)
    mx = (int(max_size) if max_size is not None else int(mine.sizes.max().item())) if mine.n else 0
    if solo:
        ns, totals, mxs = [mine.n], [mine.total], [mx]
    else:
        meta = _gather_flat(torch.tensor([mine.n, mine.total, mx], dtype=torch.int64, device=device), world)
        meta = meta.view(world, 3).tolist()
        ns, totals, mxs = [m[0] for m in meta], [m[1] for m in meta], [m[2] for m in meta]
    log_b = log_b_for(max(max(mxs), 1))
    if solo:
        lay = ops.build(mine, log_b, None, "own")
        out = torch.zeros((n_genomes, n_genomes), dtype=torch.int32, device=device)
        res.counts = res.matrix = out
        if pipelined and ani_ones is not None and ani_host is not None and n_genomes and hasattr(ops, "count_range"):
            # rows of tile rows [0, I) are final once those tile rows are counted
            # (the row-major upper triangle; the mirror halves come from earlier
            # rows): each part's ANI rows are computed and copied into ani_host on a
            # copy stream while the next part's tiles are counted
            n, nb = n_genomes, (n_genomes + TILE - 1) // TILE
            res.ani = torch.empty((n, n), dtype=torch.float64, device=device)
            copy = _copy_stream(device)
            flat_d, flat_h = res.ani.view(-1), ani_host.view(-1)
            for I0, I1 in _row_parts(nb):
                ops.count_range(n, log_b, lay, _tiles_before(I0, nb), _tiles_before(I1, nb), out)
                r0, r1 = I0 * TILE, min(n, I1 * TILE)
                ops.ani_rows(out, n, r0, r1, ani_ones, res.ani)
                ev = torch.cuda.Event()
                ev.record()
                copy.wait_event(ev)
                with torch.cuda.stream(copy):
                    flat_h[r0 * n:r1 * n].copy_(flat_d[r0 * n:r1 * n], non_blocking=True)
            torch.cuda.current_stream().wait_stream(copy)
            return res
        if n_genomes:
            ops.count(n_genomes, log_b, lay, 0, lay, 0, None, out)
        if ani_ones is not None:
            res.ani = ops.ani_matrix(out, n_genomes, ani_ones)
            if ani_host is not None:
                ani_host.view(-1).copy_(res.ani.view(-1), non_blocking=True)
        return res
    # rank 0's group bounds, shared by every layout (blocks of different ranks
    # are joined bucket by bucket)
    gb = ops.bounds(mine, log_b) if rank == 0 else ops.bounds_like(log_b)
    gb = _broadcast(gb, 0, world)
    local, remote = tile_plan_by_peer(n_genomes, world, rank)
    T = len(local) + sum(len(r) for r in remote)
    parts = torch.zeros((max(T, 1), TILE, TILE), dtype=torch.int32, device=device)
    wait = _exchange_start(mine, ns, totals, world, rank)
    own = ops.build(mine, log_b, gb, "own") if mine.n else None
    if len(local):  # the rank's own tiles while the peers' sketches travel
        ops.count(n_genomes, log_b, own, g0 // TILE, own, g0 // TILE, local, parts[:len(local)])
    off = len(local)
    srcs = [None] * world
    for q in range(world):
        srcs[q] = wait(q)
        tq = remote[q]
        if q == rank or not len(tq):
            continue
        lq = ops.build(srcs[q], log_b, gb, ("peer", q))
        bq = block_shard(n_genomes, world, q)[1] // TILE
        if rank < q:
            ops.count(n_genomes, log_b, own, g0 // TILE, lq, bq, tq, parts[off:off + len(tq)])
        else:
            ops.count(n_genomes, log_b, lq, bq, own, g0 // TILE, tq, parts[off:off + len(tq)])
        off += len(tq)
    res.tiles = np.concatenate([local] + list(remote)).reshape(-1, 2)
    res.counts = parts[:T]
    if ani_ones is not None:
        sizes_all = torch.cat([srcs[q].sizes for q in range(world)])
        res.ani = ops.ani_tiles(res.tiles, res.counts, sizes_all, n_genomes, ani_ones)
    if dst is None:
        return res
    plans = [tile_plan(n_genomes, world, q) for q in range(world)]
    counts = [len(pl[0]) + len(pl[1]) for pl in plans]
    pad = torch.zeros((max(max(counts), 1), TILE, TILE), dtype=torch.int32, device=device)
    pad[:T] = res.counts
    gathered = _gather_tiles(pad, world, None if dst == "all" else dst)
    if gathered is None:
        return res
    tiles = np.concatenate([np.concatenate(pl) for pl in plans]).reshape(-1, 2)
    got = torch.cat([gathered[q, :counts[q]] for q in range(world)])
    out = torch.zeros((n_genomes, n_genomes), dtype=torch.int32, device=device)
    res.matrix = place_tiles(out, tiles, got, n_genomes)
    return res


_COPY_STREAMS = {}


def _copy_stream(device):
    """A high-priority side stream per device for device-to-host copies (HIP maps
    streams onto four hardware queues; a normal-priority copy stream can land on
    the compute stream's queue and wait behind its kernels: DESIGN.md §6)."""
    key = str(device)
    if key not in _COPY_STREAMS:
        lo, hi = torch.cuda.Stream.priority_range()
        _COPY_STREAMS[key] = torch.cuda.Stream(device=device, priority=hi)
    return _COPY_STREAMS[key]


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


class GpuJoinOps:
    """The kernels of all_vs_all_join on the GPU through libsks: a context `ctx`
    and the k-mer width (ew = 1: u64, 2: 128-bit).  Layout buffers persist per
    build key across calls of the same shape; the context's HIP stream is
    ordered after torch's current stream before its kernels and torch's after
    them, so a context on any stream works with the collectives on torch's."""

    def __init__(self, ctx, ew=1):
        import sksffi
        self.sksffi, self.ctx, self.ew = sksffi, ctx, ew
        self.bufs, self.tile_cache, self.keep = {}, {}, {}

    def bounds_like(self, log_b):
        return torch.empty((self.sksffi.join_layout_groups(log_b) + 1) * self.ew, dtype=torch.int64, device="cuda")

    def bounds(self, src, log_b):
        b = self.bounds_like(log_b)
        _ctx_waits_for_torch(self.ctx)
        self.ctx.join_layout_bounds(src.data.data_ptr(), src.starts.data_ptr(), src.sizes.data_ptr(), src.n, log_b,
                                    b.data_ptr(), elem_words=self.ew)
        _torch_waits_for_ctx(self.ctx)
        self.keep["bounds"] = src
        return b

    def build(self, src, log_b, gb, key):
        nb = (src.n + TILE - 1) // TILE
        shape = (max(src.total, 1), log_b, max(nb, 1))
        if self.bufs.get(key, (None,))[0] != shape:
            BW = self.sksffi.join_layout_boff_words(log_b)
            self.bufs[key] = (shape, (torch.empty(shape[0] * self.ew, dtype=torch.int64, device="cuda"),
                                      torch.empty(shape[0], dtype=torch.int64, device="cuda"),
                                      torch.zeros(shape[2] * BW, dtype=torch.int32, device="cuda"),
                                      torch.zeros(shape[2] + 1, dtype=torch.int64, device="cuda")))
        lay = self.bufs[key][1]
        if src.n:
            _ctx_waits_for_torch(self.ctx)  # the buffers' previous readers, the source's writers
            self.ctx.join_layout_build(src.data.data_ptr(), src.starts.data_ptr(), src.sizes.data_ptr(), src.n,
                                       log_b, *(t.data_ptr() for t in lay), stat=False, total=src.total,
                                       bounds=gb.data_ptr() if gb is not None else None, elem_words=self.ew)
            _torch_waits_for_ctx(self.ctx)
        self.keep[key] = (src, gb)  # alive until torch's stream is past the build
        return lay

    def _tiles(self, tiles):
        key = tiles.tobytes()  # the plan repeats every step: upload it once
        if key not in self.tile_cache:
            if len(self.tile_cache) > 64:
                self.tile_cache.clear()
            self.tile_cache[key] = torch.from_numpy(np.array(tiles, dtype=np.int32)).reshape(-1, 2).to("cuda")
        return self.tile_cache[key]

    def count(self, n, log_b, rows, r_blk0, cols, c_blk0, tiles, out):
        _ctx_waits_for_torch(self.ctx)
        if tiles is None:
            self.ctx.intersect_layout_tiles(n, log_b, *(t.data_ptr() for t in rows), 0, 0, 0,
                                            self.sksffi.intersect_sym_tiles(n), False, out.data_ptr(),
                                            elem_words=self.ew)
        else:
            tl = self._tiles(tiles)
            self.ctx.intersect_layout_pair_tiles(n, log_b, [t.data_ptr() for t in rows], r_blk0,
                                                 [t.data_ptr() for t in cols], c_blk0, tl.data_ptr(), 0,
                                                 tl.shape[0], out.dim() == 3, out.data_ptr(), elem_words=self.ew)
        _torch_waits_for_ctx(self.ctx)

    def count_range(self, n, log_b, lay, tile_begin, tile_end, out):
        """Upper-triangle tiles [tile_begin, tile_end) of one layout, counts added
        to the dense n x n matrix out (both halves)."""
        _ctx_waits_for_torch(self.ctx)
        self.ctx.intersect_layout_tiles(n, log_b, *(t.data_ptr() for t in lay), 0, 0, tile_begin, tile_end,
                                        False, out.data_ptr(), elem_words=self.ew)
        _torch_waits_for_ctx(self.ctx)

    def ani_rows(self, counts, n, r0, r1, k, ani):
        _ctx_waits_for_torch(self.ctx)
        self.ctx.ani_rows(counts.data_ptr(), n, r0, r1, k, ani.data_ptr())
        _torch_waits_for_ctx(self.ctx)

    def ani_matrix(self, counts, n, k):
        ani = torch.empty((n, n), dtype=torch.float64, device="cuda")
        _ctx_waits_for_torch(self.ctx)
        self.ctx.ani_matrix(counts.data_ptr(), n, k, ani.data_ptr())
        _torch_waits_for_ctx(self.ctx)
        return ani

    def ani_tiles(self, tiles, packed, sizes, n, k):
        out = torch.empty((len(tiles), 2, TILE, TILE), dtype=torch.float64, device="cuda")
        if len(tiles):
            tl = self._tiles(tiles)
            sz = sizes.to(device="cuda", dtype=torch.int32).contiguous()
            _ctx_waits_for_torch(self.ctx)
            self.ctx.ani_tiles(packed.data_ptr(), tl.data_ptr(), len(tiles), n, sz.data_ptr(), k, out.data_ptr())
            _torch_waits_for_ctx(self.ctx)
            self.keep["ani_sizes"] = sz
        return out


def sketches_of(ss, ew=None):
    """Sketches (zero-copy device views) of a SketchSet, or an empty set for None."""
    if ss is None:
        e = ew or 1
        return Sketches(torch.zeros(0, dtype=torch.int64, device="cuda"),
                        torch.zeros(0, dtype=torch.int32, device="cuda"), e)
    d, st, sz = ss.device_tensors(torch.cuda.current_device())
    return Sketches(d, sz, ss.elem_words, starts=st)


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
